"""Probe (diagnostic, GPU): constraint-solver iterations per step (mjData.solver_niter) of a bench
workload.  Usage: niter.py [c2|c3|c4|c5] [PGS|CG|Newton] [envs]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
solver = sys.argv[2] if len(sys.argv) > 2 else None
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
if cfg == "c2":
    xml, base = bench.ref_scene_xml(sensors=False)
else:
    path = ROOT / "scenes" / (dict(c3="arm7_lidar", c4="mobile_base", c5="arm_boxes")[cfg] + ".xml")
    xml, base = path.read_text(), str(path.parent)
if solver:
    xml = bench.with_solver(xml, solver)
model = sim.Model.from_string(xml, base)
b = sim.Batch(model, n)
b.set(sim.FIELD_QPOS, synth.initial_qpos(model, np.arange(n)))
period = 10
table = torch.from_numpy(synth.ctrl_table(model, np.arange(n), 12, period).astype(np.float32)).cuda()
hist = np.zeros(64, dtype=np.int64)
for p in range(10):
    b.set_ctrl_device(table[p].data_ptr())
    for k in range(period):
        b.step(1)
        if p >= 3:
            it = b.get(sim.FIELD_SOLVER_NITER).ravel().astype(int)
            hist += np.bincount(np.minimum(it, 63), minlength=64)
print(cfg, solver or "scene", "niter histogram (index = iterations):", {i: int(c) for i, c in enumerate(hist) if c})
