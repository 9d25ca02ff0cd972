# Quick GPU check after a kernel change: GPU tests, then bench lines (no CPU baseline) for $CFGS,
# then the phase ablation for $ABL (optional).  Every GPU step has its own time limit.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for c in ${CFGS:-c3 c4}; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/q_$c.json 2> gpurun_out/q_$c.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/q_$c.json')); r=d['roofline']; print('$c', round(d['value']/1e6,2), 'M', round(r['kernel_ms'],4), r.get('step_kernel_ms'))"
done
for c in ${ABL:-}; do CFG=$c bash scripts/gpu_ablate.sh || exit $?; done
