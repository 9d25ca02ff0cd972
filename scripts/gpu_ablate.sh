# Phase ablation of the C3 bench (diagnostic only: MRS_DIAG_SKIP bit 0 sensors, 1 collision,
# 2 constraints), kernel ms per 10-step launch from the bench's own HIP events
set -u
for sk in 0 1 2 4 7; do
  echo "== skip $sk"
  MRS_DIAG_SKIP=$sk timeout -k 10 200 python bench.py --config ${CFG:-c3} --steps 100 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['roofline']['kernel_ms'],4), round(d['value']/1e6,1))" || exit $?
done
