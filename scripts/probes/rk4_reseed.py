"""Probe (diagnostic, GPU): the re-seeded RK4 comparison step by step (per-step worst env)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "oracle"))
from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402
import binding  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "mobile_base"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 32
integ = sys.argv[3] if len(sys.argv) > 3 else "RK4"
xml = (ROOT / "scenes" / f"{name}.xml").read_text().replace('integrator="implicitfast"', f'integrator="{integ}"')
model = sim.Model.from_string(xml, str(ROOT / "scenes"))
period, settle, steps = 10, 20, 60
envs = np.arange(n)
qpos0 = synth.initial_qpos(model, envs)
table = synth.ctrl_table(model, envs, (steps + settle) // period + 1, period)
orc = [binding.OracleData(model) for _ in envs]
ref = [binding.OracleData(model) for _ in envs]
for e, d in enumerate(orc):
    d.qpos[:] = qpos0[e]
for t in range(settle):
    for e, d in enumerate(orc):
        if t % period == 0:
            d.ctrl[:] = table[t // period, e]
        d.step()
b = sim.Batch(model, n)
for t in range(settle, settle + steps):
    for e, (d, r) in enumerate(zip(orc, ref)):
        if t % period == 0:
            d.ctrl[:] = table[t // period, e]
        for k in ("qpos", "qvel", "qacc_warmstart", "ctrl"):
            getattr(r, k)[:] = getattr(d, k).astype(np.float32)
    b.set(sim.FIELD_QPOS, np.array([r.qpos for r in ref]))
    b.set(sim.FIELD_QVEL, np.array([r.qvel for r in ref]))
    b.set(sim.FIELD_QACC_WARMSTART, np.array([r.qacc_warmstart for r in ref]))
    b.set(sim.FIELD_CTRL, np.array([r.ctrl for r in ref]))
    b.step(1)
    for d, r in zip(orc, ref):
        r.step(); d.step()
    v = b.get(sim.FIELD_QVEL); vr = np.array([r.qvel for r in ref])
    err = np.max(np.abs(v - vr) / np.maximum(np.abs(vr), 1), axis=1)
    nc = b.get(sim.FIELD_NCON)[:, 0].astype(int); nr = np.array([r.ncon for r in ref])
    e = int(np.argmax(err))
    if err[e] > 1e-5 or (nc != nr).any():
        print(t, "worst env", e, "err", err[e], "ncon gpu/orc", nc[e], nr[e], "flips", int(np.sum(nc != nr)),
              "bad envs", np.nonzero(err > 1e-5)[0].tolist()[:12])
print("done")
