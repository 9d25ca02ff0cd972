"""MPR contact polish diagnostics (oracle only, CPU), on states of the MPR test scene
(tests/test_gpu_mesh.py MPR_SCENE): per contact, the polished normal against MPR's (ORC_NO_POLISH=1)
and against a brute-force minimisation of the support function of A - B over the unit sphere.
  python scripts/diag_mpr.py [n_states]"""
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PATHS = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
sys.path[:0] = PATHS
import numpy as np  # noqa: E402

STATES = f"""
import sys; sys.path[:0] = {PATHS!r}
import numpy as np
from mujoco_ros2_simulation_amd import sim, synth
import binding
from test_gpu_mesh import MPR_SCENE
model = sim.Model.from_string(MPR_SCENE)
d = binding.OracleData(model)
d.qpos[:] = synth.initial_qpos(model, np.arange(1))[0]
Q, V = [], []
for t in range(75 + int(sys.argv[2])):
    d.step()
    if t >= 75: Q.append(d.qpos.copy()); V.append(d.qvel.copy())
np.savez(sys.argv[1], q=np.array(Q), v=np.array(V))
"""
CONTACTS = f"""
import sys, json; sys.path[:0] = {PATHS!r}
import numpy as np
from mujoco_ros2_simulation_amd import sim
import binding
from test_gpu_mesh import MPR_SCENE
model = sim.Model.from_string(MPR_SCENE)
z = np.load(sys.argv[1])
out = []
for q, v in zip(z["q"], z["v"]):
    e = binding.OracleData(model)
    e.qpos[:] = q; e.qvel[:] = v
    e.forward()
    g, dist, pos, frame = e.contacts()
    out.append([g.tolist(), dist.tolist(), pos.tolist(), frame[:, :3].tolist()])
print(json.dumps(out))
"""


def contacts(path, no_polish):
    env = dict(os.environ)
    env.pop("ORC_NO_POLISH", None)
    if no_polish:
        env["ORC_NO_POLISH"] = "1"
    r = subprocess.run([sys.executable, "-c", CONTACTS, path], capture_output=True, text=True, env=env, check=True)
    return json.loads(r.stdout)


def main(n):
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "states.npz")
        env = dict(os.environ, ORC_NO_POLISH="1")
        subprocess.run([sys.executable, "-c", STATES, path, str(n)], check=True, env=env)
        a, b = contacts(path, True), contacts(path, False)
    from mujoco_ros2_simulation_amd import sim
    from test_gpu_mesh import MPR_SCENE
    model = sim.Model.from_string(MPR_SCENE)
    ch, kinds = [], {}
    for ra, rb in zip(a, b):
        assert ra[0] == rb[0]
        for k, (g1, g2) in enumerate(ra[0]):
            x = float(np.max(np.abs(np.array(ra[3][k]) - np.array(rb[3][k]))))
            kind = (int(model.geom_type[g1]), int(model.geom_type[g2]))
            kinds.setdefault(kind, []).append(x)
    for kind, xs in sorted(kinds.items()):
        xs = np.array(xs)
        print(f"pair types {kind}: {len(xs)} contacts, polished on {int(np.sum(xs > 1e-12))}, "
              f"normal change max {xs.max():.2e} median {np.median(xs):.2e}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 60)


def brute(n_states=30):
    """the polished normal against a direct minimisation of h(n) = h_A(n) + h_B(-n) (scipy
    Nelder-Mead on the sphere from MPR's normal) on the same states"""
    from scipy.optimize import minimize
    from mujoco_ros2_simulation_amd import sim
    import binding
    from test_gpu_mesh import MPR_SCENE
    model = sim.Model.from_string(MPR_SCENE)
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "states.npz")
        subprocess.run([sys.executable, "-c", STATES, path, str(n_states)], check=True,
                       env=dict(os.environ, ORC_NO_POLISH="1"))
        z = np.load(path)
        a, b = contacts(path, True), contacts(path, False)

    def support(g, gpos, gmat, n):
        t, sz = model.geom_type[g], model.geom_size[g]
        R = gmat[g].reshape(3, 3)
        l = R.T @ n
        if t in (2, 3):
            p = sz[0] * l / np.linalg.norm(l)
            if t == 3:
                p[2] += sz[1] if l[2] >= 0 else -sz[1]
        elif t == 4:
            tt = sz ** 2 * l
            p = tt / np.sqrt(tt @ l)
        elif t == 7:
            mid = model.geom_dataid[g]
            va, nh, ha = model.mesh_vertadr[mid], model.mesh_hullnum[mid], model.mesh_hulladr[mid]
            V = model.mesh_vert[va + model.mesh_hull[ha:ha + nh]]
            p = V[np.argmax(V @ l)]
        else:
            raise ValueError(t)
        return gpos[g] + R @ p

    worst_h = worst_n = 0.0
    for i, (q, v) in enumerate(zip(z["q"], z["v"])):
        e = binding.OracleData(model)
        e.qpos[:] = q
        e.qvel[:] = v
        e.forward()
        _, _, gpos, gmat = e.kinematics()
        for k, (g1, g2) in enumerate(a[i][0]):
            if model.geom_type[g1] == 0:
                continue
            h = lambda n: (support(g1, gpos, gmat, n) - support(g2, gpos, gmat, -n)) @ n  # noqa: E731
            n_mpr, n_pol = np.array(a[i][3][k]), np.array(b[i][3][k])

            def f(x):
                nn = np.array([np.cos(x[0]) * np.cos(x[1]), np.sin(x[0]) * np.cos(x[1]), np.sin(x[1])])
                return h(nn)
            x0 = [np.arctan2(n_mpr[1], n_mpr[0]), np.arcsin(np.clip(n_mpr[2], -1, 1))]
            r = minimize(f, x0, method="Nelder-Mead", options={"xatol": 1e-12, "fatol": 1e-15, "maxiter": 20000})
            nb = np.array([np.cos(r.x[0]) * np.cos(r.x[1]), np.sin(r.x[0]) * np.cos(r.x[1]), np.sin(r.x[1])])
            worst_h = max(worst_h, h(n_pol) - r.fun)
            worst_n = max(worst_n, np.max(np.abs(nb - n_pol)))
            if h(n_pol) - r.fun > 1e-9 or np.max(np.abs(nb - n_pol)) > 1e-4:
                print("mismatch", i, g1, g2, model.geom_type[g1], model.geom_type[g2], "h_pol - h* =", h(n_pol) - r.fun,
                      "h_mpr - h* =", h(n_mpr) - r.fun, "|n_pol - n*| =", np.max(np.abs(nb - n_pol)))
    print(f"brute force: h(polished) - min h <= {worst_h:.2e}; |n_polished - argmin| <= {worst_n:.2e}")
