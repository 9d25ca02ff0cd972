# HBM traffic of the step kernel from PMC counters, one counter group per pass (MI355X_MICROARCH.md:
# FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).  Timing-free; bounded.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || exit $?
ls -R gpurun_out/pmc_fetch gpurun_out/pmc_write
