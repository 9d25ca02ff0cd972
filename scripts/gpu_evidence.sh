# Round evidence on one GPU box, in two calls (each under gpurun's limit):
#   PART=A: GPU tests, smoke, one bench line per config (with its CPU baseline), the 1080-beam line
#   PART=B: rocprofv3 kernel statistics per config, then PMC passes (FETCH_SIZE, WRITE_SIZE, fp32 VALU
#           flops, SQ) per config -- each pass its own run, as MI355X_MICROARCH.md prescribes
# Every GPU step has its own time limit; the script stops at the first failure (no retries).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
CFGS=${CFGS:-"c3 c2 c4 c5 c3m"}
if [ "${PART:-A}" = A ]; then
  timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
  timeout -k 10 120 python bench.py --config c1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err || exit $?
  for c in $CFGS; do
    timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
  done
  timeout -k 10 300 python bench.py --config c3 --scene scenes/arm7_lidar1080.xml --no-cpu-baseline > gpurun_out/bench_c3_1080.json 2> gpurun_out/bench_c3_1080.err || exit $?
  # extra lines: C5 and C4 under MuJoCo's default solver (Newton)
  timeout -k 10 300 python bench.py --config c5 --solver Newton --steps 40 --warmup 4 --no-cpu-baseline > gpurun_out/bench_c5_newton.json 2> gpurun_out/bench_c5_newton.err || exit $?
  timeout -k 10 300 python bench.py --config c4 --solver Newton --no-cpu-baseline > gpurun_out/bench_c4_newton.json 2> gpurun_out/bench_c4_newton.err || exit $?
  exit 0
fi
[ "${SKIP_STATS:-0}" = 1 ] || for c in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_$c -o run -- python3 bench.py --config $c --no-cpu-baseline > gpurun_out/rocprof_$c.log 2>&1 || exit $?
done
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
for c in $CFGS; do
  ps=5; [ $c = c4 ] && ps=200; [ $c = c3m ] && ps=20
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$c -o run -- python3 bench.py --config $c --steps $ps --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_$c.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$c -o run -- python3 bench.py --config $c --steps $ps --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_$c.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_flops_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_flops_$c.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_sq_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq_$c.log 2>&1 || exit $?
done
