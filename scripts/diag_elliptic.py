"""re-seeded elliptic steps on the GPU for solver x impratio (diagnostic)"""
import sys
sys.path[:0] = ["tests", "oracle"]
from test_gpu_elliptic import elliptic_scene
from test_gpu_solvers import _reseeded

for scene, solver, imp in (("arm_boxes", "Newton", 1.0), ("arm_boxes", "CG", 3.0), ("arm_boxes", "CG", 1.0),
                           ("mobile_base", "CG", 1.0), ("mobile_base", "PGS", 1.0), ("arm_boxes", "PGS", 1.0)):
    m = elliptic_scene(scene, solver, imp)
    wq, wv, ncon, flips, un = _reseeded(m, 8, 12)
    print(scene, solver, imp, f"qpos {wq:.2e} qvel {wv:.2e} flips {flips} ncon {ncon.mean():.1f}", flush=True)
