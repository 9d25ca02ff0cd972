# A/B: library variants (AB="libmrs.so libmrs_x.so ...") x lane-group widths (GROUPS_TO_RUN)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab_groups.log
for v in ${AB:-libmrs.so}; do
  for g in ${GROUPS_TO_RUN:-16 32 64}; do
    echo "== $v group $g" >> gpurun_out/ab_groups.log
    MRS_LIB=$PWD/mujoco_ros2_simulation_amd/$v MRS_GROUP=$g timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline >> gpurun_out/ab_groups.log 2>&1 || exit $?
  done
done
echo done
