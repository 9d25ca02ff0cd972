# Phase ablation of C3 (MRS_DIAG_SKIP bits: 1 sensors, 2 collision, 4 constraints), kernel ms only,
# plus one memory-instruction PMC pass.  Each GPU step time-bounded; stop at first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ablate.txt
for skip in 0 1 2 4 6 7; do
  MRS_DIAG_SKIP=$skip timeout -k 10 120 python bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/abl_$skip.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/abl_$skip.json')); print('skip $skip', round(d['roofline']['kernel_ms'],4))" >> gpurun_out/ablate.txt
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA --kernel-trace --output-format csv -d gpurun_out/pmc_sq2_c3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq2_c3.log 2>&1 || exit $?
cat gpurun_out/ablate.txt
