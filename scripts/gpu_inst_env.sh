# Dynamic instruction mix of one bench config's step kernel under a list of environment settings
# (phase ablation by MRS_DIAG_SKIP): one rocprofv3 --pmc pass per setting with 8 SQ counters.
#   CFG=c3 ENVS="- MRS_DIAG_SKIP=1" bash scripts/gpu_inst_env.sh
# Per-wave-step counts land in gpurun_out/inst_<cfg>_<tag>.json (scripts/inst_summary.py).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
CNT=${CNT:-"SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY"}
for e in ${ENVS:--}; do
  tag=$(echo "$e" | tr '=,/' '___')
  if [ "$e" = "-" ]; then envset=""; else envset=$(echo "$e" | tr ',' ' '); fi
  rm -rf gpurun_out/pmc_inst_${CFG}_$tag
  env $envset timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d gpurun_out/pmc_inst_${CFG}_$tag -o run -- python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_inst_${CFG}_$tag.log 2>&1 || exit $?
  python3 scripts/inst_summary.py gpurun_out/pmc_inst_${CFG}_$tag gpurun_out/inst_${CFG}_$tag.json "$e" || exit $?
done
