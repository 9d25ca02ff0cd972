# Round evidence on one GPU box, in two calls (each under gpurun's limit):
#   PART=A: GPU tests, smoke, one bench line per variant (with its CPU baseline for the plain configs)
#   PART=B: rocprofv3 kernel statistics per variant, then PMC passes (FETCH_SIZE, WRITE_SIZE, fp32 VALU
#           flops, SQ) per variant -- each pass its own run, as MI355X_MICROARCH.md prescribes
# A variant is KEY:CFG:EXTRA -- KEY is bench.py's variant_key (the file key of its bench line and
# counter summaries), EXTRA the --solver / --scene arguments (commas for spaces).  Every GPU step has
# its own time limit; the script stops at the first failure (no retries).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"c3:c3: c2:c2: c4:c4: c5:c5: c3m:c3m: c5_newton:c5:--solver,Newton c4_newton:c4:--solver,Newton c3_arm7_lidar1080:c3:--scene,scenes/arm7_lidar1080.xml"}
if [ "${PART:-A}" = A ]; then
  if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
  fi
  timeout -k 10 120 python bench.py --config c1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err || exit $?
  for v in $VARIANTS; do
    key=${v%%:*}; rest=${v#*:}; cfg=${rest%%:*}; extra=$(echo ${rest#*:} | tr ',' ' ')
    cpu=""; [ -n "$extra" ] && cpu="--no-cpu-baseline"
    timeout -k 10 300 python bench.py --config $cfg $extra $cpu > gpurun_out/bench_$key.json 2> gpurun_out/bench_$key.err || exit $?
  done
  exit 0
fi
for v in $VARIANTS; do
  key=${v%%:*}; rest=${v#*:}; cfg=${rest%%:*}; extra=$(echo ${rest#*:} | tr ',' ' ')
  [ "${SKIP_STATS:-0}" = 1 ] || timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_$key -o run -- python3 bench.py --config $cfg $extra --no-cpu-baseline > gpurun_out/rocprof_$key.log 2>&1 || exit $?
  [ "${SKIP_PMC:-0}" = 1 ] && continue
  # (render configs: enough bench steps for several frame batches -- C4 renders every 10 bench steps)
  ps=5; [ $cfg = c4 ] && ps=40; [ $cfg = c3m ] && ps=20
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$key -o run -- python3 bench.py --config $cfg $extra --steps $ps --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_$key.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_$key -o run -- python3 bench.py --config $cfg $extra --steps $ps --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_$key.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_flops_$key -o run -- python3 bench.py --config $cfg $extra --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_flops_$key.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_sq_$key -o run -- python3 bench.py --config $cfg $extra --steps $ps --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq_$key.log 2>&1 || exit $?
done
