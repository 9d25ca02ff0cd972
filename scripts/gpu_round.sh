# Standard GPU measurement pass (run on the MI355X box via gpurun).  Every GPU step is time-bounded
# and the script stops at the first GPU failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
if [ "${AB:-}" != "" ]; then
  for v in $AB; do
    echo "== $v" >> gpurun_out/ab.log
    MRS_LIB=$PWD/mujoco_ros2_simulation_amd/$v timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline >> gpurun_out/ab.log 2>&1 || exit $?
  done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1 || exit $?
tail -3 gpurun_out/pytest_gpu.log
