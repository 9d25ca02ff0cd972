"""Environment sharding across ranks: one process per GPU, each owning a contiguous
range of global env ids; the synthetic inputs (synth.py) are keyed by global env id, so results do not
depend on the rank count.  There is no collective in the data path: torch.distributed (RCCL over xGMI
on GPUs, gloo on CPU) only times the job (barrier + max over ranks) and gathers the observations the
host consumes to rank 0."""
from __future__ import annotations

import os

import numpy as np


def env_ids(rank: int, envs_per_rank: int) -> np.ndarray:
    """global env ids owned by `rank` (weak scaling: every rank owns envs_per_rank envs)"""
    return rank * envs_per_rank + np.arange(envs_per_rank)


def spawn(nprocs: int, argv: list[str], grace: float = 10.0, poll: float = 0.1) -> int:
    """Start `nprocs` ranks of `argv` (a Python command line) as child processes with the torchrun
    environment (RANK, LOCAL_RANK = GPU index, WORLD_SIZE, MASTER_ADDR 127.0.0.1, a free port) and
    wait for them; returns the first non-zero exit code (0 if all succeed).  A rank that fails ends the
    job: its siblings (blocked in the rendezvous or a collective until the backend's timeout otherwise)
    are terminated, then killed after `grace` seconds.  The caller must not have touched the GPU: each
    child owns one device."""
    import socket
    import subprocess
    import sys
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs),
                   LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
    import time
    first_bad = 0
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            first_bad = bad[0]
            break
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(poll)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.monotonic() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return first_bad


def init(backend: str | None = None):
    """(rank, world, local_rank) from the torchrun environment; joins the process group when world > 1
    (backend 'nccl' = RCCL when GPUs are used, 'gloo' on CPU)"""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            be = backend or ("nccl" if torch.cuda.is_available() else "gloo")
            kw = {"device_id": torch.device("cuda", local)} if be == "nccl" else {}
            dist.init_process_group(be, **kw)
    return rank, world, local


def max_over_ranks(values, device="cpu"):
    """element-wise max of a list of floats over all ranks (the job time is the slowest rank's)"""
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


class ObsGather:
    """End-of-step observation gather to rank 0: every rank's [n_local, dim] rows of
    each observation field go to the root with grouped point-to-point ops (`batch_isend_irecv`: on an
    xGMI node one direct link per peer, not a ring).  Double buffered: `start(k)` returns the buffers
    of slot k % 2 to be filled (by the producer, on the current stream) and `launch()` posts the
    transfers; the next `start` of the same slot first makes the current stream wait for that slot's
    previous transfer, so the producer overlaps the one in flight.  Rank 0's gathered rows of slot k
    are `gathered(k)[f]` ([world, n_local, dim]; its own rows are filled in place)."""

    def __init__(self, n_local: int, dims: list[int], device="cpu"):
        import torch
        import torch.distributed as dist
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self._bufs = [[torch.zeros((self.world, n_local, d), device=device) for d in dims] for _ in range(2)]
        self._pending = [None, None]
        self._slot = 0

    def start(self, k: int):
        self._slot = k % 2
        for w in self._pending[self._slot] or []:
            w.wait()
        self._pending[self._slot] = None
        return [b[self.rank] for b in self._bufs[self._slot]]

    def launch(self):
        import torch.distributed as dist
        if self.world == 1:
            return
        ops = []
        for b in self._bufs[self._slot]:
            if self.rank == 0:
                ops += [dist.P2POp(dist.irecv, b[r], r) for r in range(1, self.world)]
            else:
                ops.append(dist.P2POp(dist.isend, b[self.rank], 0))
        self._pending[self._slot] = dist.batch_isend_irecv(ops)

    def gathered(self, k: int):
        for w in self._pending[k % 2] or []:
            w.wait()
        self._pending[k % 2] = None
        return self._bufs[k % 2]


def gather_rows(t, dst: int = 0):
    """concatenate every rank's [n_local, ...] tensor on rank `dst` in rank order (None elsewhere);
    equal n_local on every rank"""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())] if dist.get_rank() == dst else None
    dist.gather(t, parts, dst=dst)
    return torch.cat(parts) if parts is not None else None
