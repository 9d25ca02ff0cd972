# GPU tests, then the C3 bench twice (no CPU baseline).  Bounded; stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 ${BENCH_ARGS:-} > gpurun_out/tb_$i.json 2>/dev/null || exit $?
done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/tb_*.json')):
    d=json.load(open(f)); print(f, round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],4))
"
