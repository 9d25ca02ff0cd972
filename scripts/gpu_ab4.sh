# C4 bench of libmrs_<v>.so for v in VARIANTS, two interleaved rounds
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ab4_*.json
for i in 1 2; do
  for v in $VARIANTS; do
    MRS_LIB=$PWD/mujoco_ros2_simulation_amd/libmrs_$v.so timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 100 > gpurun_out/ab4_${v}_$i.json 2>/dev/null || exit $?
  done
done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/ab4_*.json')):
    d=json.load(open(f)); r=d['roofline']; print(f, round(d['value']/1e6,2), 'depth', round(r['kernel_ms'],4), 'step', round(r['step_kernel_ms'],4))
"
