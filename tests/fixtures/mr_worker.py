"""Rank worker for tests/test_multirank.py::test_spawn_and_obs_gather: started by shard.spawn (the
launcher bench.py --gpus N uses), joins a gloo group, steps its env shard with the CPU oracle and
gathers every period's (qpos, qvel) to rank 0 through shard.ObsGather (the double-buffered
point-to-point gather bench.py runs over RCCL); rank 0 saves the gathered rows of every period."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import binding  # noqa: E402
from mujoco_ros2_simulation_amd import shard, sim, synth  # noqa: E402

PER_RANK, PERIODS, PERIOD = 3, 4, 10


def main(out: str):
    rank, world, local = shard.init("gloo")
    assert world == int(os.environ["WORLD_SIZE"]) and local == rank
    m = sim.Model.load(ROOT / "tests" / "golden" / "ref_scenes" / "scene.xml")
    ids = shard.env_ids(rank, PER_RANK)
    q0 = synth.initial_qpos(m, ids)
    tab = synth.ctrl_table(m, ids, PERIODS, PERIOD)
    envs = [binding.OracleData(m) for _ in ids]
    for e, d in enumerate(envs):
        d.qpos[:] = q0[e]
    g = shard.ObsGather(PER_RANK, [m.nq, m.nv])
    rows = []
    for p in range(PERIODS):
        for e, d in enumerate(envs):
            d.ctrl[:] = tab[p, e]
            d.step(PERIOD)
        q, v = g.start(p)
        import torch
        q.copy_(torch.tensor(np.array([d.qpos for d in envs]), dtype=torch.float32))
        v.copy_(torch.tensor(np.array([d.qvel for d in envs]), dtype=torch.float32))
        g.launch()
        if p >= 1 and rank == 0:   # the previous period's slot, as a consumer one period behind would
            gq, gv = g.gathered(p - 1)
            rows.append(np.concatenate([gq.reshape(world * PER_RANK, -1).numpy(),
                                        gv.reshape(world * PER_RANK, -1).numpy()], axis=1).copy())
    if rank == 0:
        gq, gv = g.gathered(PERIODS - 1)
        rows.append(np.concatenate([gq.reshape(world * PER_RANK, -1).numpy(),
                                    gv.reshape(world * PER_RANK, -1).numpy()], axis=1))
        np.save(out, np.stack(rows))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
