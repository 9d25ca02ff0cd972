"""numpy restatement of the MPR steps of oracle.c mpr_penetration / step.hip mpr_penetration in a chosen
float type (diagnostics: where fp32 and fp64 MPR part ways on a given pair).
    python scripts/mpr_np.py STATE_INDEX   (states of the MPR test scene, tests/test_gpu_mesh.py)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np  # noqa: E402

from mujoco_ros2_simulation_amd import sim, synth  # noqa: E402
import binding  # noqa: E402


class Shape:
    def __init__(self, model, g, gpos, gmat, margin, F):
        self.F = F
        self.type = int(model.geom_type[g])
        self.pos = gpos[g].astype(F)
        self.mat = gmat[g].reshape(3, 3).astype(F)
        self.size = model.geom_size[g].astype(F)
        self.inflate = F(0.5 * margin)
        if self.type == 7:
            mid = model.geom_dataid[g]
            va, hn, ha = model.mesh_vertadr[mid], model.mesh_hullnum[mid], model.mesh_hulladr[mid]
            self.hull = model.mesh_vert[va + model.mesh_hull[ha:ha + hn]].astype(F)

    def support(self, d):
        F = self.F
        l = self.mat.T @ d
        z = self.size
        if self.type == 4:  # ellipsoid
            t = z * z * l
            den = np.sqrt(t @ l)
            p = t / den if den > 1e-15 else np.zeros(3, F)
        elif self.type == 2:
            n = np.sqrt(l @ l)
            p = z[0] * l / n
        elif self.type == 7:
            dots = self.hull @ l
            k = int(np.argmax(dots))  # first maximum, as the loops' strict '>'
            p = self.hull[k]
        else:
            raise NotImplementedError(self.type)
        dn = np.sqrt(d @ d)
        return (self.mat @ p + self.pos + (self.inflate * d / dn if dn > 1e-15 else 0)).astype(F)


def mpr(A, B, F, eps, trace=False):
    tol = F(1e-6)

    def sup(d):
        a = A.support(d)
        b = B.support(-d)
        return a - b

    def nrmz(v):
        return (v / np.sqrt(v @ v)).astype(F)

    p = [None] * 4
    p[0] = (A.pos - B.pos).astype(F)
    d = nrmz(-p[0])
    p[1] = sup(d)
    if p[1] @ d <= 0:
        return None
    d = np.cross(p[0], p[1])
    d = nrmz(d)
    p[2] = sup(d)
    if p[2] @ d <= 0:
        return None
    d = nrmz(np.cross(p[1] - p[0], p[2] - p[0]))
    if d @ p[0] > 0:
        p[1], p[2] = p[2], p[1]
        d = -d
    for it in range(50):
        p[3] = sup(d)
        if p[3] @ d <= 0:
            return None
        if np.cross(p[1], p[3]) @ p[0] < -eps:
            p[2] = p[3]
        elif np.cross(p[3], p[2]) @ p[0] < -eps:
            p[1] = p[3]
        else:
            break
        d = nrmz(np.cross(p[1] - p[0], p[2] - p[0]))

    def tri_n():
        return nrmz(np.cross(p[2] - p[1], p[3] - p[1]))

    def expand(v4):
        x = np.cross(v4, p[0])
        if p[1] @ x > 0:
            if p[2] @ x > 0:
                p[1] = v4
            else:
                p[3] = v4
        else:
            if p[3] @ x > 0:
                p[2] = v4
            else:
                p[1] = v4

    def reach(v4, n):
        d4 = v4 @ n
        return min(d4 - p[1] @ n, d4 - p[2] @ n, d4 - p[3] @ n) <= tol

    it = 0
    while True:
        n = tri_n()
        if n @ p[1] >= 0:
            break
        v4 = sup(n)
        if v4 @ n < 0 or reach(v4, n) or it >= 50:
            return None
        expand(v4)
        it += 1
    it = 0
    while True:
        n = tri_n()
        v4 = sup(n)
        if trace:
            print(f"   it {it} n {np.round(n, 5)} portal {[np.round(x, 6).tolist() for x in p[1:]]}")
        if reach(v4, n) or it > 50:
            c = nearest(p[1], p[2], p[3]) if NEAREST else closest(p[1], p[2], p[3])
            depth = np.sqrt(c @ c)
            return depth, c / depth, n
        expand(v4)
        it += 1


NEAREST = True  # oracle.c / step.hip mpr_nearest (False: the barycentric closest point alone)


def nearest(a, b, c):
    n = np.cross(b - a, c - a)
    n = (n / np.sqrt(n @ n)).astype(a.dtype)
    q = (n @ a) * n
    if all(np.cross(v - u, q - u) @ n >= 0 for u, v in ((a, b), (b, c), (c, a))):
        return q
    return closest(a, b, c)


def closest(a, b, c):
    ab, ac, ap = b - a, c - a, -a
    d1, d2 = ab @ ap, ac @ ap
    if d1 <= 0 and d2 <= 0:
        return a
    bp = -b
    d3, d4 = ab @ bp, ac @ bp
    if d3 >= 0 and d4 <= d3:
        return b
    vc = d1 * d4 - d3 * d2
    if vc <= 0 and d1 >= 0 and d3 <= 0:
        return a + d1 / (d1 - d3) * ab
    cp = -c
    d5, d6 = ab @ cp, ac @ cp
    if d6 >= 0 and d5 <= d6:
        return c
    vb = d5 * d2 - d1 * d6
    if vb <= 0 and d2 >= 0 and d6 <= 0:
        return a + d2 / (d2 - d6) * ac
    va = d3 * d6 - d5 * d4
    if va <= 0 and d4 - d3 >= 0 and d5 - d6 >= 0:
        return b + (d4 - d3) / ((d4 - d3) + (d5 - d6)) * (c - b)
    denom = 1 / (va + vb + vc)
    return a + ab * vb * denom + ac * vc * denom


def main(st):
    from test_gpu_mesh import MPR_SCENE
    model = sim.Model.from_string(MPR_SCENE)
    d = binding.OracleData(model)
    d.qpos[:] = synth.initial_qpos(model, np.arange(1))[0]
    for _ in range(75 + st + 1):
        d.step()
    o = binding.OracleData(model)
    o.qpos[:] = d.qpos.astype(np.float32)
    o.qvel[:] = d.qvel.astype(np.float32)
    o.forward()
    g, dist, pos, fr = o.contacts()
    _, _, gpos, gmat = o.kinematics()
    for k in range(len(g)):
        g1, g2 = (int(x) for x in g[k])
        if (model.geom_type[g1], model.geom_type[g2]) != (4, 7):
            continue
        margin = max(model.geom_margin[g1], model.geom_margin[g2])
        print(f"contact {k}: geoms {g1} {g2} oracle n {np.round(fr[k, :3], 5)} dist {dist[k]:.4e}")
        for F, eps in ((np.float64, 1e-14), (np.float32, 1e-10)):
            A, B = Shape(model, g1, gpos, gmat, margin, F), Shape(model, g2, gpos, gmat, margin, F)
            r = mpr(A, B, F, F(eps), trace=True)
            if r is None:
                print(f"  {F.__name__}: no contact")
            else:
                print(f"  {F.__name__}: depth {r[0]:.4e} n {np.round(r[1], 5)} portal normal {np.round(r[2], 5)}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 86)
