# C3 bench at group widths 16 (default) / 32 (phases out of line) / 32 (phases inlined, libmrs_inl.so)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/g16_$i.json 2>/dev/null || exit $?
  MRS_GROUP=32 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/g32_$i.json 2>/dev/null || exit $?
  MRS_GROUP=32 MRS_LIB=$PWD/mujoco_ros2_simulation_amd/libmrs_inl.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/g32inl_$i.json 2>/dev/null || exit $?
done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/g*_*.json')):
    d=json.load(open(f)); print(f, round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],4))
"
