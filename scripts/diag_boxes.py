"""Diagnostic: boxes resting on the floor, one forward on GPU vs oracle, per solver / group width."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import binding  # noqa: E402
from mujoco_ros2_simulation_amd import sim  # noqa: E402


def scene(nbox, solver):
    bodies = "".join(f'<body pos="{0.5 * k} 0 0.0999"><freejoint/><geom type="box" size="0.1 0.1 0.1" mass="1"/></body>'
                     for k in range(nbox))
    return f'<mujoco><option solver="{solver}"/><worldbody><geom type="plane" size="0 0 1"/>{bodies}</worldbody></mujoco>'


for nbox in (4, 5, 8, 10):
    for solver in ("Newton",):
        m = sim.Model.from_string(scene(nbox, solver))
        rng = np.random.default_rng(0)
        qvel = rng.uniform(-0.3, 0.3, m.nv)
        d = binding.OracleData(m)
        d.qvel[:] = qvel
        d.forward()
        for grp in (32, 64):
            if m.nv > grp:
                continue
            os.environ["MRS_GROUP"] = str(grp)
            b = sim.Batch(m, 1)
            b.set(sim.FIELD_QVEL, qvel[None])
            b.forward()
            qa = b.get(sim.FIELD_QACC)[0]
            err = np.abs(qa - d.qacc) / np.maximum(np.abs(d.qacc), 1)
            print(f"{nbox} box {solver} G={grp} blocked={b.layout()['blocked']} ncon {int(b.get(sim.FIELD_NCON)[0,0])}/{d.ncon} "
                  f"iters {int(b.get(sim.FIELD_SOLVER_NITER)[0,0])}/{d.solver_niter} max err {err.max():.2e}")
            if err.max() > 1e-4:
                print("   gpu", np.round(qa, 4))
                print("   orc", np.round(d.qacc, 4))
            b.close()
