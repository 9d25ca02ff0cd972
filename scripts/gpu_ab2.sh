set -u; export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/ab.log
for v in ${AB}; do
  echo "== $v" >> gpurun_out/ab.log
  MRS_LIB=$PWD/mujoco_ros2_simulation_amd/$v timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline >> gpurun_out/ab.log 2>&1 || exit $?
done
