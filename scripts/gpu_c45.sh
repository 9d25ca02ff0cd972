set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 50 > gpurun_out/bench_c5q.json 2>/dev/null || exit $?
python3 -c "
import json
for f in ['gpurun_out/bench_c4.json','gpurun_out/bench_c5q.json']:
    d=json.load(open(f)); r=d['roofline']; print(f, round(d['value']/1e6,3), round(r['kernel_ms'],4), r.get('step_kernel_ms'))
"
