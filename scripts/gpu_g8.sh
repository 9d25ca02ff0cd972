set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/g16b_$i.json 2>/dev/null || exit $?
  MRS_GROUP=8 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/g8_$i.json 2>/dev/null || exit $?
done
python3 -c "
import json,glob
for f in sorted(glob.glob('gpurun_out/g8_*.json')+glob.glob('gpurun_out/g16b_*.json')):
    d=json.load(open(f)); print(f, round(d['value']/1e6,2), round(d['roofline']['kernel_ms'],4))
"
