"""Diagnostics (GPU): contact-by-contact comparison of the device and the oracle along the oracle's
trajectory of a scene (default: tests/test_gpu_mesh.py MESH_SCENE), forward from the same fp32 state;
prints the steps whose contact positions or distances differ the most."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np
from mujoco_ros2_simulation_amd import sim, synth
import binding
import test_gpu_mesh as T

model = sim.Model.from_string(getattr(T, sys.argv[1] if len(sys.argv) > 1 else "MESH_SCENE"))
d = binding.OracleData(model)
d.qpos[:] = synth.initial_qpos(model, np.arange(1))[0]
b = sim.Batch(model, 1)
worst = []
for t in range(220):
    d.step()
    if t < 80:
        continue
    q, v = d.qpos.astype(np.float32), d.qvel.astype(np.float32)
    b.set(sim.FIELD_QPOS, q[None])
    b.set(sim.FIELD_QVEL, v[None])
    b.forward()
    g, dist, pos, fr = b.contacts(0)
    r = binding.OracleData(model)
    r.qpos[:] = q
    r.qvel[:] = v
    r.forward()
    gr, dr, pr, frr = r.contacts()
    if len(g) != len(gr) or not np.array_equal(g, gr):
        print("step", t + 1, "pair lists differ", g.tolist(), gr.tolist())
        continue
    e = np.abs(pos - pr).max(axis=1) + np.abs(dist - dr) + np.abs(fr[:, :3] - frr[:, :3]).max(axis=1)
    k = int(np.argmax(e))
    worst.append((e[k], t + 1, k, g[k].tolist(), pos[k].round(5).tolist(), pr[k].round(5).tolist(),
                  float(dist[k]), float(dr[k]), fr[k, :3].round(4).tolist(), frr[k, :3].round(4).tolist()))
worst.sort(reverse=True)
for w in worst[:8]:
    print(w)
