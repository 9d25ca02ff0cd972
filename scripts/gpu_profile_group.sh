# Ablation (MRS_DIAG_SKIP) + SQ counters for one lane-group width (MRS_GROUP, default 16)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
G=${MRS_GROUP:-16}
export MRS_GROUP=$G
: > gpurun_out/ablate_g$G.log
for skip in 0 1 4 7; do
  echo "== skip $skip" >> gpurun_out/ablate_g$G.log
  MRS_DIAG_SKIP=$skip timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline >> gpurun_out/ablate_g$G.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_sq_g$G -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq_g$G.log 2>&1 || exit $?
echo done
