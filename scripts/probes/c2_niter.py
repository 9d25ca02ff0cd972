"""Probe (diagnostic, GPU): solver iterations and row counts of the C2 bench workload."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

from bench import ref_scene_xml  # noqa: E402
from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402

n, period = 4096, 10
model = sim.Model.from_string(*ref_scene_xml(sensors=False))
b = sim.Batch(model, n)
b.set(sim.FIELD_QPOS, synth.initial_qpos(model, np.arange(n)))
table = torch.from_numpy(synth.ctrl_table(model, np.arange(n), 12, period).astype(np.float32)).cuda()
for p in range(10):
    b.set_ctrl_device(table[p].data_ptr())
    for k in range(period):
        b.step(1)
        if p % 3 == 0 and k == 0:
            it = b.get(sim.FIELD_SOLVER_NITER).ravel()
            print("period", p, "niter hist", np.bincount(it.astype(int))[:20].tolist())
print("efc env0..3", [b.efc(e)["type"].tolist() for e in range(4)])
