"""Summarize a rocprofv3 SQ-counter pass of the bench command (gpurun_out/pmc_sq_<cfg>) into the
measured-VALU record bench.py reports next to the modelled roofline (roofline.valu_measured).

Counters (one pass, 8 SQ slots + GRBM): SQ_WAVES, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_WAIT_ANY,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_ACTIVE_INST_VALU, SQ_INSTS_VALU, GRBM_GUI_ACTIVE.
MI355X_MICROARCH.md (rocprofv3 PMC slots): WAIT_ANY (parked on s_waitcnt / barrier), WAIT_INST_ANY
(issue stall) and ACTIVE_INST_ANY partition WAVE_CYCLES; the SQ cycle counters count quad-cycles.
Derived per launch of the dominant kernel:
  wait_frac        = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  issue_frac       = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  valu_issue_frac  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (share of a wave's life issuing VALU)
  valu_tflops_upper= SQ_INSTS_VALU x 64 lanes x 2 flops / kernel time (every VALU instruction
                     counted as a full-wave FMA: an upper bound on the achieved VALU flop rate)
  valu_frac_upper  = valu_tflops_upper / 157.3 TF/s (fp32 VALU peak)
  waves_per_simd   = SQ_WAVES / 1024 SIMDs
Kernel time: the bench line of the same config (gpurun_out/bench_<cfg>.json, in-bench HIP events).
Usage: python scripts/sq_summary.py OUT.json cfg
"""
import csv
import re
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = Path(sys.argv[1])
# variant key (bench.py variant_key): "<cfg>[_<solver>][_<scene>]"; directories and bench lines use
# the key, the kernel and defaults its config; extra bench arguments (--solver / --scene) from $BENCH_ARGS
KEY = sys.argv[2]
CFG = KEY.split("_")[0]
EXTRA = os.environ.get("BENCH_ARGS", "")
# SQ_KERNEL=depth_kernel summarizes the frame kernel of a render config instead (its time: the bench
# line's roofline.kernel_ms, which for C4 / C3m is the frame kernel)
KERNEL = os.environ.get("SQ_KERNEL", "step_kernel")
rows = [r for r in csv.DictReader(open(ROOT / f"gpurun_out/pmc_sq_{KEY}/run_counter_collection.csv"))
        if KERNEL in r["Kernel_Name"] and not re.search(r"step_kernel<\d+, true", r["Kernel_Name"])]
per = defaultdict(lambda: defaultdict(float))
for r in rows:
    per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
disp = sorted(per, key=int)
steady = disp[1:] if len(disp) > 2 else disp
avg = {k: sum(per[d][k] for d in steady) / len(steady) for k in per[steady[0]]}
bench = json.loads((ROOT / f"gpurun_out/bench_{KEY}.json").read_text().strip().splitlines()[-1])
kms = (bench["roofline"]["kernel_ms"] if KERNEL != "step_kernel"
       else bench["roofline"].get("step_kernel_ms") or bench["roofline"]["kernel_ms"])
wc = avg["SQ_WAVE_CYCLES"]
valu_tf = avg["SQ_INSTS_VALU"] * 64 * 2 / (kms * 1e-3) / 1e12
rec = {
    "kernel": rows[0]["Kernel_Name"], "config": KEY, "launches_averaged": len(steady),
    "counters_per_launch": avg, "kernel_ms": kms,
    "wait_frac": avg["SQ_WAIT_ANY"] / wc, "issue_stall_frac": avg["SQ_WAIT_INST_ANY"] / wc,
    "issue_frac": avg["SQ_ACTIVE_INST_ANY"] / wc, "valu_issue_frac": avg["SQ_ACTIVE_INST_VALU"] / wc,
    "valu_tflops_upper": valu_tf, "valu_frac_upper": valu_tf / 157.3,
    "waves_per_simd": avg["SQ_WAVES"] / 1024,
    "command": f"rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
               f"SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -- "
               f"python3 bench.py --config {CFG} {EXTRA} --steps 5 --warmup 1 --no-cpu-baseline",
}
OUT.write_text(json.dumps(rec, indent=1) + "\n")
print(json.dumps({k: v for k, v in rec.items() if k != "counters_per_launch"}))
