"""Summarize gpurun_out ablation logs and SQ counter CSVs (per env-step figures)."""
import collections, csv, json, sys
for g in sys.argv[1:]:
    print("group", g)
    cur = None
    for line in open(f"gpurun_out/ablate_g{g}.log"):
        if line.startswith("=="): cur = line.strip()
        elif line.startswith("{"):
            d = json.loads(line); print(" ", cur, round(d["value"] / 1e6, 2), "M", round(d["roofline"]["kernel_ms"], 3), "ms")
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/pmc_sq_g{g}/run_counter_collection.csv")):
        if "step_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    envsteps = 8192 * 10
    for k, v in sorted(agg.items()):
        a = sum(v) / len(v)
        print(f"  {k:22s} {a:14.0f}  per env-step {a / envsteps:10.1f}")
