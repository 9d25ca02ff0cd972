# A/B of the C4 frame kernel: for each library in LIBS (cur = libmrs.so, else libmrs_<name>.so) the
# frames alone (--render-every 10: one 2048-frame batch per 10-step launch) and the default C4 line.
#   LIBS="head cur" bash scripts/gpu_depth_ab.sh
export TMPDIR=/tmp; mkdir -p gpurun_out
for l in ${LIBS:-cur}; do
  lib=mujoco_ros2_simulation_amd/libmrs_$l.so; [ $l = cur ] && lib=mujoco_ros2_simulation_amd/libmrs.so
  MRS_LIB=$lib timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --render-every 10 --steps 40 > gpurun_out/d10_$l.json 2> gpurun_out/d10_$l.err || exit $?
  MRS_LIB=$lib timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline > gpurun_out/d_$l.json 2> gpurun_out/d_$l.err || exit $?
  python -c "import json; a=json.load(open('gpurun_out/d10_$l.json')); b=json.load(open('gpurun_out/d_$l.json')); print('$l', 'alone', round(a['roofline']['kernel_ms'],3), 'ms', round(a['value']/1e6,2), 'M |', 'c4', round(b['value']/1e6,2), 'M depth', round(b['roofline']['kernel_ms'],3), 'step', round(b['roofline'].get('step_kernel_ms') or 0,4))"
done
