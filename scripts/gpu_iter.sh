# Iteration pass: GPU tests, C3/C4 bench lines, phase profiles of C3 (and C5 when PHASE_C5=1).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
MRS_LIB=$PWD/mujoco_ros2_simulation_amd/libmrs_timing.so timeout -k 10 120 python scripts/phase_profile.py scenes/arm7_lidar.xml 8192 5 > gpurun_out/phase_c3.json 2>&1 || exit $?
if [ "${PHASE_C5:-0}" = "1" ]; then
  MRS_LIB=$PWD/mujoco_ros2_simulation_amd/libmrs_timing.so timeout -k 10 120 python scripts/phase_profile.py scenes/arm_boxes.xml 8192 3 > gpurun_out/phase_c5.json 2>&1 || exit $?
fi
cut -c1-400 gpurun_out/bench_c3.json gpurun_out/bench_c4.json gpurun_out/phase_c3.json
