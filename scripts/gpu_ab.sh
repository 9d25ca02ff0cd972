# A/B + ablation run on the GPU box (timing only; each step bounded)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
: > gpurun_out/ab.log
for v in libmrs.so libmrs_w8.so; do
  echo "== $v" >> gpurun_out/ab.log
  MRS_LIB=$PWD/mujoco_ros2_simulation_amd/$v timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline >> gpurun_out/ab.log 2>&1 || echo "rc=$?" >> gpurun_out/ab.log
done
for sk in 1 2 4 7; do
  echo "== skip $sk" >> gpurun_out/ab.log
  MRS_DIAG_SKIP=$sk timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline >> gpurun_out/ab.log 2>&1 || echo "rc=$?" >> gpurun_out/ab.log
done
tail -3 gpurun_out/pytest_gpu.log
