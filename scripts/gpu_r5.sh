# One GPU call: the GPU tests (PYTEST_K selects; ALL=1 runs every -m gpu test, no -x), then bench lines
# (no CPU baseline) for CFGS with optional MRS_LIB variants in LIBS.  Every GPU step has its own time
# limit and the script stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -q -m gpu -s --timeout 200 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_k.log 2>&1
  rc=$?; grep -E "passed|failed|worst|scene|Error|assert" gpurun_out/pytest_k.log | tail -12
  # test failures (1) still run the benches; a crash, abort or time limit ends the call
  [ $rc -gt 1 ] && exit $rc
fi
if [ "${ALL:-0}" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
  rc=$?; tail -12 gpurun_out/pytest_all.log
  [ $rc -gt 1 ] && exit $rc
fi
for c in ${CFGS:-}; do
  for l in ${LIBS:-cur}; do
    lib=mujoco_ros2_simulation_amd/libmrs_$l.so; [ $l = cur ] && lib=mujoco_ros2_simulation_amd/libmrs.so
    MRS_LIB=$lib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_${c}_$l.json 2> gpurun_out/b_${c}_$l.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/b_${c}_$l.json')); r=d['roofline']; print('$c', '$l', round(d['value']/1e6,3), 'M', round(r['kernel_ms'],4), r.get('step_kernel_ms'))"
  done
done
