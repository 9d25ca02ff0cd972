# One GPU call: bench lines for CFG under a list of environment settings (A/B of runtime switches).
#   CFG=c4 ENVS="MRS_SPREAD=0 MRS_SPREAD=1 MRS_DEPTH_ORDER=0" bash scripts/gpu_ab_env.sh
# ("-" runs the defaults).  Every bench has its own time limit; the script stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in ${ENVS:--}; do
  tag=$(echo "$e" | tr '=,/' '___')
  if [ "$e" = "-" ]; then envset=""; else envset=$(echo "$e" | tr ',' ' '); fi
  env $envset timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${CFG}_$tag.json 2> gpurun_out/ab_${CFG}_$tag.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/ab_${CFG}_$tag.json')); r=d['roofline']; print('$CFG', '$e', round(d['value']/1e6,3), 'M', round(r['kernel_ms'],4), r.get('step_kernel_ms'))"
done
