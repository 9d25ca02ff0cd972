"""Diagnostic: GPU vs oracle contact lists from GPU-stepped states (tests/test_gpu_parity.py
test_contact_list_bit_exact).  python scripts/diag_contacts.py [steps]"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import binding  # noqa: E402
from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
m = sim.Model.load(ROOT / "scenes" / "arm_boxes.xml")
n = 4
b = sim.Batch(m, n)
b.set(sim.FIELD_QPOS, synth.initial_qpos(m, np.arange(n)))
b.set(sim.FIELD_CTRL, synth.ctrl_table(m, np.arange(n), 1, 10)[0])
b.step(steps)
qs = b.get(sim.FIELD_QPOS)
b.forward()
for e in range(n):
    g, dist, pos, frame = b.contacts(e)
    d = binding.OracleData(m)
    d.qpos[:] = qs[e]
    d.forward()
    gr, dr, pr, fr = d.contacts()
    same = g.shape == gr.shape and np.array_equal(g, gr)
    print(f"env {e}: gpu {len(g)} oracle {len(gr)} same={same}")
    if not same:
        for i in range(max(len(g), len(gr))):
            a = f"{g[i].tolist()} d {dist[i]:+.3e} p {np.round(pos[i], 4)}" if i < len(g) else "-"
            o = f"{gr[i].tolist()} d {dr[i]:+.3e} p {np.round(pr[i], 4)}" if i < len(gr) else "-"
            print(f"  {i:2d} gpu {a} | orc {o}")
