"""Summarize rocprofv3 PMC passes (gpurun_out/pmc_fetch_<cfg>, pmc_write_<cfg>) of the bench command
into a per-launch HBM traffic record for bench.py's roofline.traffic.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports half of the bytes of wide coalesced streaming reads, so it is doubled here;
WRITE_SIZE is taken as is.
Usage: python scripts/pmc_summary.py OUT.json [cfg]
  cfg c2 / c3 / c5: the fused multi-step launches (step_kernel<G, false>); c4 / c3m: the depth kernel.
"""
import csv
import re
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
# variant key (bench.py variant_key): "<cfg>[_<solver>][_<scene>]"; directories and bench lines use
# the key, the kernel and defaults its config; extra bench arguments (--solver / --scene) from $BENCH_ARGS
KEY = (sys.argv[2] if len(sys.argv) > 2 else "c3")
CFG = KEY.split("_")[0]
EXTRA = os.environ.get("BENCH_ARGS", "")
KERNEL = "depth_kernel" if CFG in ("c4", "c3m") else "step_kernel"


def per_launch(name: str) -> tuple[float, str, int]:
    d = ROOT / f"gpurun_out/pmc_{name}_{KEY}"
    if not d.exists():
        d = ROOT / f"gpurun_out/pmc_{name}"
    rows = [r for r in csv.DictReader(open(d / "run_counter_collection.csv"))
            if KERNEL in r["Kernel_Name"] and (KERNEL != "step_kernel" or not re.search(r"step_kernel<\d+, true", r["Kernel_Name"]))]
    vals = [float(r["Counter_Value"]) for r in rows]
    steady = vals[1:] if len(vals) > 2 else vals  # drop the first (cold caches)
    return sum(steady) / len(steady), rows[0]["Kernel_Name"], len(steady)


fetch_kib, kname, n1 = per_launch("fetch")
write_kib, _, n2 = per_launch("write")
steps = {"c4": 200, "c3m": 20}.get(CFG, 5)  # C4: 20 depth frames, C3m: 2
rec = {
    "kernel": kname,
    "config": KEY,
    "launches_averaged": min(n1, n2),
    "fetch_size_kib_raw": fetch_kib,
    "write_size_kib": write_kib,
    "fetch_bytes": 2 * fetch_kib * 1024,
    "write_bytes": write_kib * 1024,
    "traffic_bytes_per_launch": 2 * fetch_kib * 1024 + write_kib * 1024,
    "correction": "FETCH_SIZE x2 (gfx950 half-count, MI355X_MICROARCH.md HBM section); WRITE_SIZE as is",
    "command": f"rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-trace -- python3 bench.py --config {CFG} {EXTRA} "
               f"--steps {steps} --warmup 1 --no-cpu-baseline",
}
out = Path(sys.argv[1])
out.write_text(json.dumps(rec, indent=1) + "\n")
print(json.dumps(rec))
