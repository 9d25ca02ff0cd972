"""Executed fp32 VALU work of the dominant kernel from a rocprofv3 counter pass of the bench command
(gpurun_out/pmc_flops_<cfg>), next to the modelled SURVEY.md §8(d) figure.

Counters (one pass): SQ_INSTS_VALU_FMA_F32, SQ_INSTS_VALU_ADD_F32, SQ_INSTS_VALU_MUL_F32,
SQ_INSTS_VALU_TRANS_F32, SQ_INSTS_VALU_FLOPS_FP32, SQ_WAVES, GRBM_GUI_ACTIVE.
Per launch of the dominant kernel (step_kernel<G, false> or depth_kernel_v2):
  flops_fullwave  = 64 x (2 FMA + ADD + MUL + TRANS) instructions: every fp32 VALU instruction counted
                    as 64 active lanes (an upper bound: idle lanes of a 16-lane group are counted)
  flops_counter   = SQ_INSTS_VALU_FLOPS_FP32 (gfx950: "FLOPS per instruction on float 32"), reported raw:
                    it reads ~2% of flops_fullwave on C3, so its unit (per-SE sampling, per-instruction
                    rather than per-lane counting) is not the lane-flop count this needs, and it is not used
  flops_executed  = flops_fullwave (an upper bound: lanes idle in a 16-lane group's dof phases count)
  flops_executed_per_env_step = flops_executed / (envs x physics steps per launch)
Kernel time: the bench line of the same config (gpurun_out/bench_<cfg>.json, in-bench HIP events).
Usage: python scripts/flops_summary.py OUT.json cfg [envs] [steps_per_launch]
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
ENVS = int(sys.argv[3]) if len(sys.argv) > 3 else {"c2": 4096, "c3": 8192, "c3m": 8192, "c4": 2048, "c5": 8192}[CFG]
STEPS = int(sys.argv[4]) if len(sys.argv) > 4 else 10
COUNTERS = ["SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32",
            "SQ_INSTS_VALU_FLOPS_FP32", "SQ_WAVES", "GRBM_GUI_ACTIVE"]
rows = [r for r in csv.DictReader(open(ROOT / f"gpurun_out/pmc_flops_{KEY}/run_counter_collection.csv"))
        if "step_kernel" in r["Kernel_Name"] and not re.search(r"step_kernel<\d+, true", r["Kernel_Name"])]
per = defaultdict(lambda: defaultdict(float))
for r in rows:
    per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
disp = sorted(per, key=int)
steady = disp[1:] if len(disp) > 2 else disp
avg = {k: sum(per[d][k] for d in steady) / len(steady) for k in per[steady[0]]}
bench = json.loads((ROOT / f"gpurun_out/bench_{KEY}.json").read_text().strip().splitlines()[-1])
kms = bench["roofline"].get("step_kernel_ms") or bench["roofline"]["kernel_ms"]
full = 64 * (2 * avg["SQ_INSTS_VALU_FMA_F32"] + avg["SQ_INSTS_VALU_ADD_F32"] + avg["SQ_INSTS_VALU_MUL_F32"]
             + avg["SQ_INSTS_VALU_TRANS_F32"])
cnt = avg.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0)
executed = full
units = ENVS * STEPS
tf = executed / (kms * 1e-3) / 1e12
rec = {
    "kernel": rows[0]["Kernel_Name"], "config": KEY, "launches_averaged": len(steady),
    "counters_per_launch": avg, "kernel_ms": kms, "env_steps_per_launch": units,
    "flops_fullwave_per_launch": full, "flops_counter_per_launch": cnt,
    "flops_executed_per_launch": executed, "flops_executed_per_env_step": executed / units,
    "flops_counter_over_fullwave": cnt / full if full else None,
    "executed_tflops": tf, "frac_executed": tf / 157.3,
    "command": f"rocprofv3 --pmc {' '.join(COUNTERS)} --kernel-trace -- "
               f"python3 bench.py --config {CFG} {EXTRA} --steps 5 --warmup 1 --no-cpu-baseline",
}
OUT.write_text(json.dumps(rec, indent=1) + "\n")
print(json.dumps({k: v for k, v in rec.items() if k != "counters_per_launch"}))
