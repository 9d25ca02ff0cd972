"""Synthetic inputs for parity runs and benchmarks (SURVEY.md §8d "Synthetic inputs").

Counter-based Philox4x32-10 (Salmon et al., SC'11; Random123), key = (0xC0FFEE, 0), counter =
(env, index, stream, 0), so every env's draws depend only on its *global* env id: CPU oracle and
GPU see identical inputs for any sharding over GPUs.

  initial state : qpos = qpos0 + U(-0.1, 0.1) per hinge/slide dof (stream 1), qvel = 0
  actions       : ctrl[e, t, u] = c0[u] + A[e,u] sin(2 pi f[e,u] t h + phi[e,u])   (stream 0)
                  A ~ U(0, 0.5*half ctrlrange or 0.5), f ~ U(0.2, 2) Hz, phi ~ U(0, 2 pi),
                  held (zero-order hold) for `period` physics steps, i.e. the 500 Hz physics /
                  50 Hz controller ratio of the reference test config (test/config/controllers.yaml:3)
"""
from __future__ import annotations

import numpy as np

from . import sim

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
KEY = (0xC0FFEE, 0)


def philox4x32(counter: np.ndarray, key=KEY, rounds: int = 10) -> np.ndarray:
    """counter: uint32 array [..., 4] -> uint32 [..., 4]."""
    c = np.asarray(counter, dtype=np.uint32)
    c0, c1, c2, c3 = (c[..., i].astype(np.uint64) for i in range(4))
    k0, k1 = np.uint32(key[0]), np.uint32(key[1])
    mask = np.uint64(0xFFFFFFFF)
    for r in range(rounds):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        n0 = (hi1 ^ c1 ^ np.uint64(k0)) & mask
        n2 = (hi0 ^ c3 ^ np.uint64(k1)) & mask
        c0, c1, c2, c3 = n0, lo1, n2, lo0
        k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def uniforms(env_ids: np.ndarray, n_idx: int, stream: int) -> np.ndarray:
    """[len(env_ids), n_idx, 4] uniforms in [0, 1) (24-bit mantissa, exact in fp32 and fp64)."""
    e = np.asarray(env_ids, dtype=np.uint32)
    ctr = np.zeros((e.size, n_idx, 4), dtype=np.uint32)
    ctr[..., 0] = e[:, None]
    ctr[..., 1] = np.arange(n_idx, dtype=np.uint32)[None, :]
    ctr[..., 2] = stream
    x = philox4x32(ctr)
    return (x >> np.uint32(8)).astype(np.float64) * (1.0 / (1 << 24))


def initial_qpos(model: "sim.Model", env_ids: np.ndarray) -> np.ndarray:
    q = np.tile(model.qpos0, (len(env_ids), 1))
    u = uniforms(env_ids, max(model.nq, 1), 1)[..., 0]
    for j in range(model.njnt):
        if model.jnt_type[j] in (sim.JNT_HINGE, sim.JNT_SLIDE):
            a = model.jnt_qposadr[j]
            q[:, a] += -0.1 + 0.2 * u[:, a]
    return q


def action_params(model: "sim.Model", env_ids: np.ndarray):
    u = uniforms(env_ids, max(model.nu, 1), 0)[:, :model.nu]
    c0 = np.zeros(model.nu)
    half = np.full(model.nu, 0.5)
    for a in range(model.nu):
        j = model.actuator_trnid[a, 0]
        if model.actuator_type(a) == sim.ACT_POSITION:
            c0[a] = model.qpos0[model.jnt_qposadr[j]]
        if model.actuator_ctrllimited[a]:
            lo, hi = model.actuator_ctrlrange[a]
            c0[a] = 0.5 * (lo + hi) if model.actuator_type(a) != sim.ACT_POSITION else c0[a]
            half[a] = 0.5 * 0.5 * (hi - lo)
    A = u[..., 0] * half[None, :]
    f = 0.2 + 1.8 * u[..., 1]
    phi = 2 * np.pi * u[..., 2]
    return c0, A, f, phi


def ctrl_table(model: "sim.Model", env_ids: np.ndarray, n_periods: int, period: int,
               t0_step: int = 0) -> np.ndarray:
    """[n_periods, n_envs, nu] ctrl values, one row per zero-order-hold period."""
    c0, A, f, phi = action_params(model, env_ids)
    h = model.timestep
    t = (t0_step + np.arange(n_periods) * period) * h
    return c0[None, None, :] + A[None] * np.sin(2 * np.pi * f[None] * t[:, None, None] + phi[None])
