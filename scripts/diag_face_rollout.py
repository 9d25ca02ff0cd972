"""Diagnostics (GPU): where the mesh scene's rollout (tests/test_gpu_mesh.py MESH_SCENE) first differs
between the device and the oracle -- per step, each env's contact pair list on both sides, free-running
from the same start; prints the first differing steps with the pairs and distances."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np
from mujoco_ros2_simulation_amd import sim, synth
import binding
from test_gpu_mesh import MESH_SCENE

restate = int(sys.argv[1]) if len(sys.argv) > 1 else 0
model = sim.Model.from_string(MESH_SCENE)
model.set_restate(restate)
n, steps = 4, 200
q0 = synth.initial_qpos(model, np.arange(n))
b = sim.Batch(model, n)
b.set(sim.FIELD_QPOS, q0)
orc = []
for e in range(n):
    d = binding.OracleData(model)
    d.qpos[:] = q0[e]
    orc.append(d)
shown = 0
for t in range(steps):
    b.step(1)
    for d in orc:
        d.step()
    q = b.get(sim.FIELD_QPOS)
    for e in range(n):
        # contacts of this step's forward: re-run forward on copies at the pre-step state is not
        # available on the device, so compare the pair lists of a forward at the post-step state
        r = binding.OracleData(model)
        r.qpos[:] = q[e]
        r.qvel[:] = b.get(sim.FIELD_QVEL, e, 1)[0]
        r.forward()
        gr, dr, _, _ = r.contacts()
        err = np.max(np.abs(q[e] - orc[e].qpos))
        if shown < 12 and (err > 1e-5):
            gd = orc[e].contacts()[0]
            print(f"step {t + 1} env {e}: |q - q_oracle| {err:.2e}; oracle-at-device-state ncon {len(gr)}, "
                  f"oracle ncon {len(gd)}")
            print("   pairs at device state:", gr.tolist(), np.round(dr, 5).tolist())
            print("   oracle pairs:         ", gd.tolist())
            shown += 1
b.close()
