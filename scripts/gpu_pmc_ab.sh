# HBM traffic A/B of library variants on one bench config (FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes, per MI355X_MICROARCH.md): VARIANTS="name ..." ("base" = libmrs.so), CFG (not c4).
# Summaries via scripts/pmc_summary.py into gpurun_out/pmc_ab_<cfg>_<variant>.json.
set -u
export TMPDIR=/tmp
cfg=${CFG:-c5}
for v in ${VARIANTS}; do
  lib=mujoco_ros2_simulation_amd/libmrs_$v.so; [ $v = base ] && lib=mujoco_ros2_simulation_amd/libmrs.so
  for c in fetch write; do
    C=$(echo $c | tr a-z A-Z)_SIZE
    MRS_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_${c}_${cfg}$v -o run -- python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_${c}_${cfg}$v.log 2>&1 || exit $?
  done
  python3 scripts/pmc_summary.py gpurun_out/pmc_ab_${cfg}_$v.json ${cfg}$v > /dev/null || exit $?
  echo "== $v $(python3 -c "import json; d=json.load(open('gpurun_out/pmc_ab_${cfg}_$v.json')); print(round(d['fetch_bytes']/1e6,1), 'MB fetch', round(d['write_bytes']/1e6,1), 'MB write per launch')")"
done
