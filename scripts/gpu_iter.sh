# Iteration loop on one GPU box: a subset of the GPU tests (PYTEST_K), bench lines for CFGS (no CPU
# baseline) and, when PHASE is set, the phase profile of that scene with the timing build
# (mujoco_ros2_simulation_amd/libmrs_timing.so).  Every GPU step has its own time limit; the script
# stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_iter.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_iter.log; tail -4 gpurun_out/pytest_iter.log
  [ $rc -ne 0 ] && exit $rc
fi
for c in ${CFGS:-}; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/it_$c.json 2> gpurun_out/it_$c.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/it_$c.json')); r=d['roofline']; print('$c', round(d['value']/1e6,3), 'M', round(r['kernel_ms'],4), r.get('step_kernel_ms'))"
done
if [ -n "${PHASE:-}" ]; then
  MRS_LIB=mujoco_ros2_simulation_amd/libmrs_timing.so timeout -k 10 200 python scripts/phase_profile.py $PHASE > gpurun_out/phase_iter.json 2>gpurun_out/phase_iter.err || exit $?
  cat gpurun_out/phase_iter.json
fi
if [ -n "${PMC:-}" ]; then
  for c in $PMC; do
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/it_fetch_$c.log 2>&1 || exit $?
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/it_write_$c.log 2>&1 || exit $?
    python scripts/pmc_summary.py gpurun_out/pmc_iter_$c.json $c > /dev/null 2>&1 || exit $?
    python -c "import json; d=json.load(open('gpurun_out/pmc_iter_$c.json')); print('$c traffic GB', round(d['traffic_bytes_per_launch']/1e9,3), 'fetch', round(d['fetch_bytes']/1e9,3), 'write', round(d['write_bytes']/1e9,3))"
  done
fi
