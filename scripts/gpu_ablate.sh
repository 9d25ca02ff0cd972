# Phase ablation (MRS_DIAG_SKIP bits: 1 sensors, 2 collision, 4 constraints) + SQ instruction/cycle
# counters of the step kernel.  Each GPU step time-bounded; stop at first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ablate.log
for skip in 0 1 2 4 6 7; do
  echo "== skip $skip" >> gpurun_out/ablate.log
  MRS_DIAG_SKIP=$skip timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline >> gpurun_out/ablate.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --kernel-trace --output-format csv -d gpurun_out/pmc_sq2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq2.log 2>&1 || exit $?
echo done
