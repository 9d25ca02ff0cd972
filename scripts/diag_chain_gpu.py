import sys
sys.path[:0] = ["/root/repo", "/root/repo/oracle", "/root/repo/tests"]
import numpy as np
from mujoco_ros2_simulation_amd import sim, synth
import binding
from test_gpu_equality import scene
model = scene("PGS")
n, steps = 4, 1000
q0 = synth.initial_qpos(model, np.arange(n))
tab = synth.ctrl_table(model, np.arange(n), steps // 10 + 1, 10)
b = sim.Batch(model, n)
b.set(sim.FIELD_QPOS, q0)
gq = []
for p in range(steps // 10):
    b.set(sim.FIELD_CTRL, tab[p]); b.step(10); gq.append(b.get(sim.FIELD_QPOS).copy())
for e in [2]:
    ds = [binding.OracleData(model) for _ in range(2)]
    for d in ds: d.qpos[:] = q0[e]
    for p in range(steps // 10):
        for i, d in enumerate(ds):
            d.ctrl[:] = tab[p, e]
            for _ in range(10):
                d.step()
                if i: d.qpos[:] = d.qpos.astype(np.float32); d.qvel[:] = d.qvel.astype(np.float32)
        if p % 10 == 9:
            print(p * 10 + 10, "err", np.abs(gq[p][e, :3] - ds[0].qpos[:3]).max(), "sens", np.abs(ds[1].qpos[:3] - ds[0].qpos[:3]).max(), "ncon", ds[0].ncon, "q", np.round(ds[0].qpos[:3], 4))
