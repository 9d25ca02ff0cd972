"""re-seeded elliptic steps on the GPU for solver x impratio (diagnostic)"""
import sys
sys.path[:0] = [".", "tests", "oracle"]
from test_gpu_elliptic import elliptic_scene
from test_gpu_solvers import _reseeded

for scene, solver, imp in (("arm_boxes", "Newton", 1.0), ("arm_boxes", "CG", 3.0), ("arm_boxes", "CG", 1.0),
                           ("mobile_base", "CG", 1.0), ("mobile_base", "PGS", 1.0), ("arm_boxes", "PGS", 1.0)):
    m = elliptic_scene(scene, solver, imp)
    wq, wv, ncon, flips, un = _reseeded(m, 8, 12)
    print(scene, solver, imp, f"qpos {wq:.2e} qvel {wv:.2e} flips {flips} ncon {ncon.mean():.1f}", flush=True)

import numpy as np
from mujoco_ros2_simulation_amd import sim
import binding
for scene in ("arm_boxes", "mobile_base"):
    m = elliptic_scene(scene, "CG")
    d = binding.OracleData(m)
    d.step(30)
    b = sim.Batch(m, 1)
    for f, v in ((sim.FIELD_QPOS, d.qpos), (sim.FIELD_QVEL, d.qvel), (sim.FIELD_QACC_WARMSTART, d.qacc_warmstart),
                 (sim.FIELD_CTRL, d.ctrl)):
        if len(v):
            b.set(f, v.astype(np.float32)[None])
    r = binding.OracleData(m)
    for k in ("qpos", "qvel", "qacc_warmstart", "ctrl"):
        getattr(r, k)[:] = getattr(d, k).astype(np.float32)
    b.step(1)
    r.step()
    print(scene, "CG niter gpu", b.get(sim.FIELD_SOLVER_NITER)[0, 0], "oracle", r.solver_niter,
          "qvel err", np.max(np.abs(b.get(sim.FIELD_QVEL)[0] - r.qvel)) / max(1, np.max(np.abs(r.qvel))), flush=True)
    b.close()
