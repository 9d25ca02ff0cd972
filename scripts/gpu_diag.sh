# Diagnostics pass: GPU tests, C3 A/B against a variant library (VARIANT=name -> libmrs_<name>.so),
# one SQ-counter PMC pass of the C3 bench.  Bounded; stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/ab_base_$i.json 2>/dev/null || exit $?
  MRS_LIB=$PWD/mujoco_ros2_simulation_amd/libmrs_${VARIANT}.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/ab_var_$i.json 2>/dev/null || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_sq_c3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq_c3.log 2>&1 || exit $?
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/ab_*.json')):
    d=json.load(open(f)); print(f, round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],4))
"
