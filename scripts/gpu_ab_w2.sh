# A/B: 2-wave vs default 4-wave G=16 workgroups on C3 and C4 (timing only; each step bounded)
export TMPDIR=/tmp; mkdir -p gpurun_out
: > gpurun_out/ab_w2.log
for v in libmrs.so libmrs_w2.so; do
  for c in c3 c4; do
    echo "== $v $c" >> gpurun_out/ab_w2.log
    MRS_LIB=$PWD/mujoco_ros2_simulation_amd/$v timeout -k 10 150 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline >> gpurun_out/ab_w2.log 2>&1 || exit $?
  done
done
cat gpurun_out/ab_w2.log | cut -c1-200
