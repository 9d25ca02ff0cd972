"""binned vs per-pixel mesh frames: the differing pixels against the oracle's render (diagnostic)"""
import os
import sys
sys.path[:0] = [".", "tests", "oracle"]
import numpy as np
from mujoco_ros2_simulation_amd import sim
from test_gpu_mesh import _mesh_robot, _mesh_robot_states
import binding

model = _mesh_robot("640 480")
q = _mesh_robot_states(model, n=8)
out = {}
for key in ("bin", "v2"):
    if key == "v2":
        os.environ["MRS_DEPTH_V2"] = "1"
    b = sim.Batch(model, 8)
    b.set(sim.FIELD_QPOS, q)
    b.forward()
    out[key] = b.render_depth(0, 0, 8)
    b.close()
db, dv = out["bin"], out["v2"]
for e in range(8):
    bad = np.argwhere(db[e] != dv[e])
    if len(bad) == 0:
        continue
    d = binding.OracleData(model)
    d.qpos[:] = q[e]
    d.forward()
    ref = d.render_depth(0)
    rb = np.abs(db[e] - ref)[db[e] != dv[e]]
    rv = np.abs(dv[e] - ref)[db[e] != dv[e]]
    print(f"env {e}: {len(bad)} differ; bin closer to oracle on {np.mean(rb < rv):.3f}, v2 closer {np.mean(rv < rb):.3f}; "
          f"bin>v2 on {np.mean(db[e][db[e] != dv[e]] > dv[e][db[e] != dv[e]]):.3f}; max |bin-ref| {rb.max():.2e} |v2-ref| {rv.max():.2e}")
    for (r, c) in bad[:6]:
        print(f"   px ({r},{c}) bin {db[e][r, c]:.7f} v2 {dv[e][r, c]:.7f} oracle {ref[r, c]:.7f}")
