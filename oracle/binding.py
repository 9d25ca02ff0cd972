"""TEST INFRASTRUCTURE ONLY: ctypes binding of the fp64 CPU oracle (oracle/oracle.c).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker; the
product (mujoco_ros2_simulation_amd/libmrs.so) never imports it.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liboracle.so"


class OrcData(C.Structure):
    _fields_ = [("qpos", C.POINTER(C.c_double)), ("qvel", C.POINTER(C.c_double)), ("ctrl", C.POINTER(C.c_double)),
                ("qfrc_applied", C.POINTER(C.c_double)), ("qacc_warmstart", C.POINTER(C.c_double)),
                ("time", C.c_double),
                ("qacc", C.POINTER(C.c_double)), ("qfrc_actuator", C.POINTER(C.c_double)),
                ("sensordata", C.POINTER(C.c_double)),
                ("warning", C.c_int * 4), ("ncon", C.c_int), ("nefc", C.c_int), ("solver_niter", C.c_int),
                ("ws", C.c_void_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            import subprocess
            subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
        L = C.CDLL(str(LIB_PATH))
        P = C.POINTER(C.c_double)
        L.orc_make_data.restype = C.POINTER(OrcData)
        L.orc_make_data.argtypes = [C.c_void_p]
        L.orc_free_data.argtypes = [C.POINTER(OrcData)]
        L.orc_reset.argtypes = [C.c_void_p, C.POINTER(OrcData), C.c_int]
        L.orc_step.argtypes = [C.c_void_p, C.POINTER(OrcData)]
        L.orc_forward.argtypes = [C.c_void_p, C.POINTER(OrcData)]
        L.orc_mass_matrix.argtypes = [C.c_void_p, C.POINTER(OrcData), P]
        L.orc_bias_vel.argtypes = [C.c_void_p, C.POINTER(OrcData), P]
        L.orc_kinematics.argtypes = [C.c_void_p, C.POINTER(OrcData), P, P, P, P]
        L.orc_ray.restype = C.c_double
        L.orc_ray.argtypes = [C.c_void_p, C.POINTER(OrcData), P, P, C.c_int, C.POINTER(C.c_int)]
        L.orc_render_depth.argtypes = [C.c_void_p, C.POINTER(OrcData), C.c_int, C.POINTER(C.c_float)]
        L.orc_render_rgbd.argtypes = [C.c_void_p, C.POINTER(OrcData), C.c_int, C.c_void_p, C.c_void_p]
        L.orc_contacts.argtypes = [C.POINTER(OrcData), C.c_int, C.POINTER(C.c_int), P, P, P]
        L.orc_candidate_pairs.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_smooth.argtypes = [C.c_void_p, C.POINTER(OrcData), P, P]
        L.orc_efc.argtypes = [C.POINTER(OrcData), C.c_int, C.c_int, C.POINTER(C.c_int), P, P, P, P, P]
        L.orc_rollout.restype = C.c_double
        L.orc_rollout.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, P, P, C.c_int, P, P]
        _lib = L
    return _lib


def _dp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OracleData:
    """One environment stepped by the oracle on a Model (mujoco_ros2_simulation_amd.sim.Model)."""

    def __init__(self, model):
        self.model = model
        self._mv = C.byref(model.view)
        self._d = lib().orc_make_data(self._mv)

    def _arr(self, name: str, n: int) -> np.ndarray:
        ptr = getattr(self._d.contents, name)
        return np.ctypeslib.as_array(ptr, shape=(max(n, 1),))[:n]

    @property
    def qpos(self): return self._arr("qpos", self.model.nq)
    @property
    def qvel(self): return self._arr("qvel", self.model.nv)
    @property
    def ctrl(self): return self._arr("ctrl", self.model.nu)
    @property
    def qfrc_applied(self): return self._arr("qfrc_applied", self.model.nv)
    @property
    def qacc_warmstart(self): return self._arr("qacc_warmstart", self.model.nv)
    @property
    def qacc(self): return self._arr("qacc", self.model.nv)
    @property
    def qfrc_actuator(self): return self._arr("qfrc_actuator", self.model.nv)
    @property
    def sensordata(self): return self._arr("sensordata", self.model.nsensordata)
    @property
    def time(self): return self._d.contents.time
    @property
    def warning(self): return list(self._d.contents.warning)
    @property
    def ncon(self): return self._d.contents.ncon
    @property
    def nefc(self): return self._d.contents.nefc
    @property
    def solver_niter(self): return self._d.contents.solver_niter

    def reset(self, key: int = -1):
        lib().orc_reset(self._mv, self._d, key)

    def step(self, n: int = 1):
        for _ in range(n):
            lib().orc_step(self._mv, self._d)

    def forward(self):
        lib().orc_forward(self._mv, self._d)

    def mass_matrix(self) -> np.ndarray:
        M = np.zeros(self.model.nv * self.model.nv)
        lib().orc_mass_matrix(self._mv, self._d, _dp(M))
        return M.reshape(self.model.nv, self.model.nv)

    def bias_vel(self) -> np.ndarray:
        """d qfrc_bias / d qvel at the current state (after forward), [nv, nv]"""
        dB = np.zeros(self.model.nv * self.model.nv)
        lib().orc_bias_vel(self._mv, self._d, _dp(dB))
        return dB.reshape(self.model.nv, self.model.nv)

    def kinematics(self):
        m = self.model
        xpos, xquat = np.zeros(3 * m.nbody), np.zeros(4 * m.nbody)
        gpos, gmat = np.zeros(3 * max(m.ngeom, 1)), np.zeros(9 * max(m.ngeom, 1))
        lib().orc_kinematics(self._mv, self._d, _dp(xpos), _dp(xquat), _dp(gpos), _dp(gmat))
        return (xpos.reshape(-1, 3), xquat.reshape(-1, 4), gpos[:3 * m.ngeom].reshape(-1, 3),
                gmat[:9 * m.ngeom].reshape(-1, 9))

    def ray(self, pnt, vec, bodyexclude: int = -1):
        gid = C.c_int(-1)
        p = np.ascontiguousarray(pnt, dtype=np.float64)
        v = np.ascontiguousarray(vec, dtype=np.float64)
        d = lib().orc_ray(self._mv, self._d, _dp(p), _dp(v), bodyexclude, C.byref(gid))
        return d, gid.value

    def render_depth(self, cam: int) -> np.ndarray:
        W, H = self.model.cam_resolution[cam]
        out = np.zeros((H, W), dtype=np.float32)
        lib().orc_render_depth(self._mv, self._d, cam, out.ctypes.data_as(C.POINTER(C.c_float)))
        return out

    def render_rgbd(self, cam: int) -> tuple[np.ndarray, np.ndarray]:
        W, H = self.model.cam_resolution[cam]
        depth = np.zeros((H, W), dtype=np.float32)
        rgb = np.zeros((H, W, 3), dtype=np.uint8)
        lib().orc_render_rgbd(self._mv, self._d, cam, depth.ctypes.data, rgb.ctypes.data)
        return depth, rgb

    def contacts(self, max_n: int = 256):
        g = np.zeros(2 * max_n, dtype=np.int32)
        dist, pos, frame = np.zeros(max_n), np.zeros(3 * max_n), np.zeros(9 * max_n)
        n = lib().orc_contacts(self._d, max_n, g.ctypes.data_as(C.POINTER(C.c_int)), _dp(dist), _dp(pos), _dp(frame))
        n = min(n, max_n)
        return g[:2 * n].reshape(-1, 2), dist[:n], pos[:3 * n].reshape(-1, 3), frame[:9 * n].reshape(-1, 9)

    def smooth(self):
        """(qacc_smooth, qfrc_smooth) of the last forward"""
        a, f = np.zeros(self.model.nv), np.zeros(self.model.nv)
        lib().orc_smooth(self._mv, self._d, _dp(a), _dp(f))
        return a, f

    def efc(self, max_n: int = 1024):
        """constraint rows of the last forward: dict of type [n], force, aref, R, pos [n], J [n, nv]"""
        nv = self.model.nv
        t = np.zeros(max_n, dtype=np.int32)
        f, a, R, p = (np.zeros(max_n) for _ in range(4))
        J = np.zeros(max_n * max(nv, 1))
        n = lib().orc_efc(self._d, nv, max_n, t.ctypes.data_as(C.POINTER(C.c_int)), _dp(f), _dp(a), _dp(R), _dp(p), _dp(J))
        n = min(n, max_n)
        return {"type": t[:n], "force": f[:n], "aref": a[:n], "R": R[:n], "pos": p[:n],
                "J": J[:n * nv].reshape(n, nv)}

    def __del__(self):
        if getattr(self, "_d", None) and _lib is not None:
            _lib.orc_free_data(self._d)
            self._d = None


def candidate_pairs(model) -> np.ndarray:
    """[npair, 2] statically admissible collision pairs by the oracle's own broad-phase filter"""
    cap = max(1, model.ngeom * model.ngeom)
    g1, g2 = np.zeros(cap, dtype=np.int32), np.zeros(cap, dtype=np.int32)
    n = lib().orc_candidate_pairs(C.byref(model.view), cap, g1.ctypes.data_as(C.POINTER(C.c_int)),
                                  g2.ctypes.data_as(C.POINTER(C.c_int)))
    return np.stack([g1[:n], g2[:n]], axis=1)


def rollout(model, qpos_init: np.ndarray, ctrl_table: np.ndarray, n_steps: int, period: int, n_threads: int):
    """CPU baseline / batch oracle: returns (seconds, qpos [n,nq], qvel [n,nv])."""
    n_envs = qpos_init.shape[0]
    qi = np.ascontiguousarray(qpos_init, dtype=np.float64)
    ct = np.ascontiguousarray(ctrl_table, dtype=np.float64)
    qo = np.zeros((n_envs, model.nq))
    vo = np.zeros((n_envs, model.nv))
    secs = lib().orc_rollout(C.byref(model.view), n_envs, n_steps, period, _dp(ct), _dp(qi), n_threads, _dp(qo), _dp(vo))
    return secs, qo, vo
