#!/bin/bash
# Copy one round's GPU evidence from gpurun_out/ (scripts/gpu_evidence.sh PART=A / B) into
# profiles/<round>/: bench lines, rocprofv3 kernel statistics, and the PMC summaries (HBM traffic,
# executed fp32 VALU flops, SQ) per variant key.  Runs here (no GPU).
#   scripts/collect_evidence.sh r06 [keys...]
set -e
round=${1:?round}; shift
keys=${@:-"c3 c2 c4 c5 c3m c5_newton c4_newton c3_arm7_lidar1080"}
root=$(cd "$(dirname "$0")/.." && pwd)
cd "$root"
mkdir -p profiles/$round
for f in pytest_gpu.log smoke.log; do [ -f gpurun_out/$f ] && cp gpurun_out/$f profiles/$round/; done
[ -f gpurun_out/bench_c1.json ] && cp gpurun_out/bench_c1.json profiles/$round/
for k in $keys; do
  [ -f gpurun_out/bench_$k.json ] && cp gpurun_out/bench_$k.json profiles/$round/bench_$k.json
  st=$(ls gpurun_out/rocprof_$k/*kernel_stats.csv 2>/dev/null | head -1 || true)
  [ -n "$st" ] && cp "$st" profiles/$round/${k}_kernel_stats.csv
  [ -d gpurun_out/pmc_fetch_$k ] && python3 scripts/pmc_summary.py profiles/$round/pmc_$k.json $k > /dev/null
  [ -d gpurun_out/pmc_flops_$k ] && python3 scripts/flops_summary.py profiles/$round/flops_$k.json $k > /dev/null
  [ -d gpurun_out/pmc_sq_$k ] && python3 scripts/sq_summary.py profiles/$round/sq_$k.json $k > /dev/null
done
ls profiles/$round
