"""Per-wave-step instruction counts of the step kernel from a rocprofv3 --pmc csv directory
(scripts/gpu_inst_env.sh): counters averaged over the kernel's launches, divided by SQ_WAVES and the
10 physics steps of a launch.  Usage: python scripts/inst_summary.py PMC_DIR OUT.json TAG"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

d, out, tag = Path(sys.argv[1]), Path(sys.argv[2]), sys.argv[3]
f = next(d.rglob("*counter_collection.csv"))
per = defaultdict(lambda: defaultdict(float))
names = {}
for row in csv.DictReader(open(f)):
    k = row["Kernel_Name"]
    if "step_kernel" not in k:
        continue
    per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    names[row["Dispatch_Id"]] = k
ids = sorted(per, key=int)
# the timed launches: skip the warm-up dispatch(es) -- take the last 5
ids = ids[-5:]
avg = {c: sum(per[i][c] for i in ids) / len(ids) for c in per[ids[0]]}
waves = avg.get("SQ_WAVES", 1.0)
res = {"tag": tag, "kernel": names[ids[0]], "launches": len(ids),
       "per_wave_step": {c: v / waves / 10 for c, v in avg.items() if c != "SQ_WAVES"}, "waves": waves}
json.dump(res, open(out, "w"), indent=1)
print(tag, {c: round(v) for c, v in res["per_wave_step"].items()})
