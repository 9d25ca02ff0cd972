# A/B of libraries on one config: for each library in LIBS (cur = libmrs.so, else libmrs_<name>.so) one
# bench line of CFG, in the order given (repeat names to interleave).
#   CFG=c4 LIBS="r6a cur r6a cur" bash scripts/gpu_lib_ab.sh
export TMPDIR=/tmp; mkdir -p gpurun_out
i=0
for l in ${LIBS:-cur}; do
  i=$((i + 1))
  lib=mujoco_ros2_simulation_amd/libmrs_$l.so; [ $l = cur ] && lib=mujoco_ros2_simulation_amd/libmrs.so
  MRS_LIB=$lib timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/lab_${CFG}_${i}_$l.json 2> gpurun_out/lab_${CFG}_${i}_$l.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/lab_${CFG}_${i}_$l.json')); r=d['roofline']; print('$CFG', '$l', round(d['value']/1e6,3), 'M', round(r['kernel_ms'],4), r.get('step_kernel_ms'))"
done
