# C5 A/B of the sparse solver inlined into the step kernel (-DMRS_SPARSE_INLINE, variant library
# libmrs_sparseinline.so) against the product build: bench lines and FETCH / WRITE passes each.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for l in cur sparseinline; do
  lib=mujoco_ros2_simulation_amd/libmrs_$l.so; [ $l = cur ] && lib=mujoco_ros2_simulation_amd/libmrs.so
  MRS_LIB=$lib timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > gpurun_out/ab_c5_$l.json 2> gpurun_out/ab_c5_$l.err || exit $?
  MRS_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_c5_$l -o run -- python3 bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_c5_$l.log 2>&1 || exit $?
  MRS_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_c5_$l -o run -- python3 bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_c5_$l.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab_c5_$l.json').read().strip().splitlines()[-1]); print('$l', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],3))"
done
