# A/B of library variants on one bench config: VARIANTS="name ..." (mujoco_ros2_simulation_amd/libmrs_<name>.so,
# "base" = libmrs.so); prints kernel ms per launch and env-steps/s
set -u
for v in ${VARIANTS}; do
  lib=mujoco_ros2_simulation_amd/libmrs_$v.so; [ $v = base ] && lib=mujoco_ros2_simulation_amd/libmrs.so
  echo "== $v"
  MRS_LIB=$lib timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps ${STEPS:-50} --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['roofline']['kernel_ms'],4), round(d['value']/1e6,2))" || exit $?
done
