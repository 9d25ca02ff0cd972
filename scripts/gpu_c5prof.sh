# C5 phase shares (timing build) and phase ablation (MRS_DIAG_SKIP), kernel ms only
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
MRS_LIB=$PWD/mujoco_ros2_simulation_amd/libmrs_timing.so timeout -k 10 120 python scripts/phase_profile.py scenes/arm_boxes.xml 8192 3 > gpurun_out/phase_c5.json 2>&1 || exit $?
: > gpurun_out/ablate_c5.txt
for skip in 0 1 2 4; do
  MRS_DIAG_SKIP=$skip timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abl5_$skip.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/abl5_$skip.json')); print('skip $skip', round(d['roofline']['kernel_ms'],3))" >> gpurun_out/ablate_c5.txt
done
cat gpurun_out/phase_c5.json gpurun_out/ablate_c5.txt
