# Full GPU evidence pass: gpu tests, smoke, bench C3/C4/C5, rocprof kernel stats per config,
# PMC traffic for C3 and C4.  Every GPU step is time-bounded; stop at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
for c in c3 c4 c5; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_$c -o run -- python3 bench.py --config $c --no-cpu-baseline > gpurun_out/rocprof_$c.log 2>&1 || exit $?
done
for c in c3 c4 c5; do
  ps=5; [ $c = c4 ] && ps=200
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$c -o run -- python3 bench.py --config $c --steps $ps --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_$c.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$c -o run -- python3 bench.py --config $c --steps $ps --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_$c.log 2>&1 || exit $?
done
tail -3 gpurun_out/pytest_gpu.log
