"""Diagnostic: one forward pass from an oracle state on the GPU and on the oracle, per solver;
prints the worst qacc mismatches (dof, GPU, oracle).  python scripts/diag_primal.py [scene] [steps]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import binding  # noqa: E402
from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "arm_boxes"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
path = ROOT / "scenes" / f"{scene}.xml"
for solver, opt in [("PGS2000", 'solver="PGS" iterations="2000" tolerance="1e-15"'),
                    ("Newton", 'solver="Newton" iterations="100"'), ("CG", 'solver="CG" iterations="100"'),
                    ("Newton1", 'solver="Newton" iterations="1"')]:
    m = sim.Model.from_string(path.read_text().replace('solver="PGS" iterations="50"', opt), str(path.parent))
    d = binding.OracleData(m)
    d.qpos[:] = synth.initial_qpos(m, np.arange(1))[0]
    d.step(steps)
    b = sim.Batch(m, 1)
    b.set(sim.FIELD_QPOS, d.qpos[None])
    b.set(sim.FIELD_QVEL, d.qvel[None])
    b.set(sim.FIELD_QACC_WARMSTART, d.qacc_warmstart[None])
    b.forward()
    d.forward()
    qa = b.get(sim.FIELD_QACC)[0]
    err = np.abs(qa - d.qacc) / np.maximum(np.abs(d.qacc), 1)
    w = np.argsort(-err)[:6]
    print(f"{solver}: ncon gpu {int(b.get(sim.FIELD_NCON)[0, 0])} oracle {d.ncon} nefc {d.nefc} iters {d.solver_niter} "
          f"gpu iters {int(b.get(sim.FIELD_SOLVER_NITER)[0, 0])} max rel err {err.max():.2e}; worst dofs " + ", ".join(f"{j}:{qa[j]:.4g}/{d.qacc[j]:.4g}" for j in w))
    b.close()
