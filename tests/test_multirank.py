"""Multi-rank path on CPU (gloo, world_size 2): env sharding by global id, gather to rank 0 and the
max-over-ranks timing give the same results as one process owning every env."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import REF_SCENE, ROOT

WORLD, PER_RANK, STEPS, PERIOD = 2, 3, 60, 10


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rollout(ids):
    sys.path.insert(0, str(ROOT / "oracle"))
    import binding
    from mujoco_ros2_simulation_amd import sim, synth
    m = sim.Model.load(REF_SCENE)
    q0 = synth.initial_qpos(m, ids)
    tab = synth.ctrl_table(m, ids, STEPS // PERIOD + 1, PERIOD)
    _, q, v = binding.rollout(m, q0, tab, STEPS, PERIOD, 1)
    return q, v


def _worker(rank, port, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    from mujoco_ros2_simulation_amd import shard
    r, w, _ = shard.init("gloo")
    assert (r, w) == (rank, WORLD)
    ids = shard.env_ids(rank, PER_RANK)
    q, v = _rollout(ids)
    allq = shard.gather_rows(torch.from_numpy(q))
    allv = shard.gather_rows(torch.from_numpy(v))
    tmax = shard.max_over_ranks([float(rank + 1), -float(rank)])
    if rank == 0:
        np.savez(out_path, q=allq.numpy(), v=allv.numpy(), tmax=np.array(tmax))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_rollout_matches_single_process(tmp_path, built):
    out = tmp_path / "gathered.npz"
    mp.spawn(_worker, args=(_free_port(), str(out)), nprocs=WORLD, join=True)
    got = np.load(out)
    q, v = _rollout(np.arange(WORLD * PER_RANK))
    assert np.array_equal(got["q"], q) and np.array_equal(got["v"], v)
    assert list(got["tmax"]) == [2.0, 0.0]


def _gather_worker(rank, port, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    from mujoco_ros2_simulation_amd import shard
    shard.init("gloo")
    g = shard.ObsGather(PER_RANK, [2, 3])
    got = []
    for k in range(4):  # four periods through the two buffer slots
        q, v = g.start(k)
        q.copy_(torch.full((PER_RANK, 2), 100.0 * k + rank))
        v.copy_(torch.arange(PER_RANK * 3, dtype=torch.float32).reshape(PER_RANK, 3) + 10 * rank + 1000 * k)
        g.launch()
        if k >= 1 and rank == 0:
            got.append([b.clone().numpy() for b in g.gathered(k - 1)])
    if rank == 0:
        got.append([b.clone().numpy() for b in g.gathered(3)])
        np.savez(out_path, **{f"p{k}_{f}": got[k][f] for k in range(4) for f in range(2)})
    dist.barrier()
    dist.destroy_process_group()


def test_observation_gather_double_buffered(tmp_path, built):
    """end-of-step observation gather with grouped point-to-point ops, world size 2 on
    gloo: rank 0 holds every rank's rows of every period, slots reused across periods"""
    out = tmp_path / "obs.npz"
    mp.spawn(_gather_worker, args=(_free_port(), str(out)), nprocs=WORLD, join=True)
    got = np.load(out)
    for k in range(4):
        q, v = got[f"p{k}_0"], got[f"p{k}_1"]
        assert q.shape == (WORLD, PER_RANK, 2) and v.shape == (WORLD, PER_RANK, 3)
        for r in range(WORLD):
            assert np.all(q[r] == 100.0 * k + r)
            assert np.array_equal(v[r], np.arange(PER_RANK * 3).reshape(PER_RANK, 3) + 10 * r + 1000 * k)


def test_env_ids_partition():
    from mujoco_ros2_simulation_amd import shard
    ids = np.concatenate([shard.env_ids(r, 5) for r in range(4)])
    assert np.array_equal(ids, np.arange(20))


def test_spawn_and_obs_gather(tmp_path, built):
    """the launcher of `bench.py --gpus N` (shard.spawn: N child ranks with the torchrun environment)
    at world size 2 on gloo, with the per-period observation gather (shard.ObsGather) that bench.py
    times for N > 1: rank 0 holds every env's (qpos, qvel) of every period, equal to one process
    stepping all envs"""
    sys.path.insert(0, str(ROOT / "tests" / "fixtures"))
    import mr_worker
    from mujoco_ros2_simulation_amd import shard, sim, synth
    import binding
    out = tmp_path / "rows.npy"
    rc = shard.spawn(2, [str(ROOT / "tests" / "fixtures" / "mr_worker.py"), str(out)])
    assert rc == 0
    got = np.load(out)
    n = 2 * mr_worker.PER_RANK
    m = sim.Model.load(REF_SCENE)
    ids = np.arange(n)
    q0 = synth.initial_qpos(m, ids)
    tab = synth.ctrl_table(m, ids, mr_worker.PERIODS, mr_worker.PERIOD)
    envs = [binding.OracleData(m) for _ in ids]
    for e, d in enumerate(envs):
        d.qpos[:] = q0[e]
    assert got.shape[0] == mr_worker.PERIODS
    for p in range(mr_worker.PERIODS):
        for e, d in enumerate(envs):
            d.ctrl[:] = tab[p, e]
            d.step(mr_worker.PERIOD)
        want = np.array([np.concatenate([d.qpos, d.qvel]) for d in envs]).astype(np.float32)
        assert np.array_equal(got[p], want), p


def test_bench_rejects_mismatched_world():
    """bench.py fails loudly when --gpus disagrees with a torchrun WORLD_SIZE"""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "does not match WORLD_SIZE=3" in r.stderr


def test_spawn_fails_fast():
    """a rank that dies ends the job: shard.spawn returns its exit code and terminates the siblings
    instead of waiting for them (they would sit in the rendezvous until the backend timeout)"""
    import time
    from mujoco_ros2_simulation_amd import shard
    code = ("import os, sys, time\n"
            "if os.environ['RANK'] == '1': sys.exit(3)\n"
            "time.sleep(300)\n")
    t0 = time.monotonic()
    rc = shard.spawn(3, ["-c", code], grace=5.0)
    assert rc == 3
    assert time.monotonic() - t0 < 60
