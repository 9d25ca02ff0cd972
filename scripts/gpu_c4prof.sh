# C4 rocprofv3 kernel stats and PMC traffic of the same command as the bench line (200 periods,
# 20 depth frames of every env), so the depth kernel's average agrees with the in-bench events
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/rocprof_c4 gpurun_out/pmc_fetch_c4 gpurun_out/pmc_write_c4
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_c4 -o run -- python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/rocprof_c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_c4 -o run -- python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/pmc_fetch_c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_c4 -o run -- python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/pmc_write_c4.log 2>&1 || exit $?
grep depth gpurun_out/rocprof_c4/run_kernel_stats.csv | cut -c1-40,200-300
cut -c1-200 gpurun_out/bench_c4.json
