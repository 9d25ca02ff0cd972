# GPU tests + C3/C5 bench lines (no CPU baseline).  Bounded; stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
cat gpurun_out/bench_c5.json gpurun_out/bench_c3.json | cut -c1-200
