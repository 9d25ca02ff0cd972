"""rangefinders of the mesh robot with and without the ray hierarchy (MRS_NO_BVH): differing rays (diagnostic)"""
import os
import sys
sys.path[:0] = [".", "tests", "oracle"]
import numpy as np
from mujoco_ros2_simulation_amd import sim
from test_gpu_mesh import _mesh_robot, _mesh_robot_states
import binding

model = _mesh_robot("160 120")
q = _mesh_robot_states(model)
out = []
for flag in (None, "1"):
    if flag:
        os.environ["MRS_NO_BVH"] = flag
    b = sim.Batch(model, len(q))
    b.set(sim.FIELD_QPOS, q)
    b.forward()
    out.append(b.get(sim.FIELD_SENSORDATA))
    b.close()
s1, s2 = out
bad = np.argwhere(s1 != s2)
print("differing", len(bad), "of", s1.size)
for e, k in bad[:12]:
    d = binding.OracleData(model)
    d.qpos[:] = q[e]
    d.forward()
    print(e, k, s1[e, k], s2[e, k], "oracle", d.sensordata[k])
