# C3 bench of the default library against VARIANTS="a b ..." (libmrs_<v>.so), two interleaved rounds
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/v_*.json
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/v_base_$i.json 2>/dev/null || exit $?
  for v in $VARIANTS; do
    MRS_LIB=$PWD/mujoco_ros2_simulation_amd/libmrs_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 ${BENCH_ARGS:-} > gpurun_out/v_${v}_$i.json 2>/dev/null || exit $?
  done
done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/v_*.json')):
    d=json.load(open(f)); print(f, round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],4))
"
