# HBM traffic of one bench config under a list of environment settings (phase ablation of traffic):
#   CFG=c5 ENVS="- MRS_DIAG_SKIP=4" bash scripts/gpu_pmc_env.sh
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (MI355X_MICROARCH.md), summaries by
# scripts/pmc_summary.py into gpurun_out/pmc_env_<cfg>_<tag>.json.  Stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in ${ENVS:--}; do
  tag=$(echo "$e" | tr '=,/' '___')
  if [ "$e" = "-" ]; then envset=""; else envset=$(echo "$e" | tr ',' ' '); fi
  for c in fetch write; do
    C=$(echo $c | tr a-z A-Z)_SIZE
    rm -rf gpurun_out/pmc_${c}_${CFG}
    env $envset timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${c}_${CFG} -o run -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${c}_${CFG}_$tag.log 2>&1 || exit $?
  done
  python3 scripts/pmc_summary.py gpurun_out/pmc_env_${CFG}_$tag.json $CFG > /dev/null || exit $?
  echo "== $e $(python3 -c "import json; d=json.load(open('gpurun_out/pmc_env_${CFG}_$tag.json')); print(round(d['fetch_bytes']/1e6,1), 'MB fetch', round(d['write_bytes']/1e6,1), 'MB write per launch')")"
done
