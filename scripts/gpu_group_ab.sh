# Group-width A/B (diagnostic): bench lines per config with MRS_GROUP forced to each width in $WIDTHS.
set -u
mkdir -p gpurun_out
for c in ${CFGS:-c4 c2}; do
  for g in ${WIDTHS:-16 32 64}; do
    MRS_GROUP=$g timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 100 > gpurun_out/gab_${c}_$g.json 2> gpurun_out/gab_${c}_$g.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/gab_${c}_$g.json')); r=d['roofline']; print('$c', 'G=$g', round(d['value']/1e6,2), 'M', round(r['kernel_ms'],4), r.get('step_kernel_ms'))"
  done
done
