# A/B of library variants in one GPU call: bench lines (no CPU baseline) per config per library,
# alternating libraries within each config.  LIBS="head new" (mujoco_ros2_simulation_amd/libmrs_<name>.so,
# "cur" = libmrs.so), CFGS="c3 c4", REPS=2.  Every GPU step has its own time limit.
set -u
mkdir -p gpurun_out
for c in ${CFGS:-c3 c4}; do
  for r in $(seq ${REPS:-2}); do
    for l in ${LIBS:-head cur}; do
      lib=mujoco_ros2_simulation_amd/libmrs_$l.so; [ $l = cur ] && lib=mujoco_ros2_simulation_amd/libmrs.so
      MRS_LIB=$lib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${c}_$l.json 2> gpurun_out/ab_${c}_$l.err || exit $?
      python -c "import json; d=json.load(open('gpurun_out/ab_${c}_$l.json')); r=d['roofline']; print('$c', '$l', round(d['value']/1e6,2), 'M', round(r['kernel_ms'],4), r.get('step_kernel_ms'))"
    done
  done
done
