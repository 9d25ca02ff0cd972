"""Probe (diagnostic, GPU): one RK4 step of a contact scene on the GPU and the oracle from the same
state, per group width.  Usage: rk4_step.py [scene] [groups]"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "oracle"))
from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402
import binding  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "mobile_base"
for integ in ["implicitfast", "RK4"]:
    xml = (ROOT / "scenes" / f"{name}.xml").read_text().replace('integrator="implicitfast"', f'integrator="{integ}"')
    for g in (sys.argv[2] if len(sys.argv) > 2 else "16,32,64").split(","):
        os.environ["MRS_GROUP"] = g
        model = sim.Model.from_string(xml, str(ROOT / "scenes"))
        n = 2
        q0 = synth.initial_qpos(model, np.arange(n)); tab = synth.ctrl_table(model, np.arange(n), 5, 10)
        orc = [binding.OracleData(model) for _ in range(n)]
        for e, d in enumerate(orc):
            d.qpos[:] = q0[e]; d.ctrl[:] = tab[0][e]; d.step(20)
        b = sim.Batch(model, n)
        for k, f in (("qpos", sim.FIELD_QPOS), ("qvel", sim.FIELD_QVEL), ("qacc_warmstart", sim.FIELD_QACC_WARMSTART), ("ctrl", sim.FIELD_CTRL)):
            b.set(f, np.stack([getattr(d, k) for d in orc]))
        b.step(1)
        for d in orc:
            d.step(1)
        gv = b.get(sim.FIELD_QVEL); gq = b.get(sim.FIELD_QPOS)
        print(integ, "G", g, "qvel err", np.abs(gv - np.stack([d.qvel for d in orc])).max(),
              "qpos err", np.abs(gq - np.stack([d.qpos for d in orc])).max(), "ncon", b.get(sim.FIELD_NCON).ravel(), [d.ncon for d in orc])
        print("   gpu qvel", np.round(gv[0], 5)); print("   orc qvel", np.round(orc[0].qvel, 5))
