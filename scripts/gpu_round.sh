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
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof.log 2>&1 || exit $?
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || exit $?
fi
tail -3 gpurun_out/pytest_gpu.log
