#!/usr/bin/env python3
"""Benchmark: batched mj_step on MI355X (BASELINE.json metric "env-steps/sec (whole node),
7-DoF arm+lidar scene").

Workload (BASELINE.json configs[2]): scenes/arm7_lidar.xml — 7-DoF arm,
360-beam rangefinder lidar, PGS — 8192 envs per GPU (weak scaling: every rank owns its own 8192
envs, global env ids rank*8192 + i, no data-path collective).  One bench "step" = one controller
period = 10 physics steps (mj_step) of every env with the period's synthetic action held (the
reference's 500 Hz physics / 50 Hz controller ratio), i.e. one fused kernel launch.  Inputs (the
whole synthetic action table) are resident in HBM before timing starts.

Prints ONE JSON line on rank 0.  Launch: `python bench.py` (1 GPU) or
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "env-steps/sec (whole node), 7-DoF arm+lidar scene at 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200, help="timed controller periods")
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--period", type=int, default=10, help="physics steps per controller period")
    p.add_argument("--envs", type=int, default=8192, help="envs per GPU")
    p.add_argument("--scene", default=str(ROOT / "scenes" / "arm7_lidar.xml"))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    p.add_argument("--config", choices=["c3", "c4", "c5"], default="c3",
                   help="c3: the BASELINE metric (default); c4: mobile base + lidar + 640x480 depth camera; "
                        "c5: contact-rich arm + 8 free boxes, PGS 50 iterations")
    p.add_argument("--render-every", type=int, default=100, help="C4: physics steps between depth frames")
    p.add_argument("--gather", action="store_true",
                   help="N>1: end-of-step observation gather, every period each rank's (qpos, qvel) to rank 0 "
                        "with grouped RCCL point-to-point ops (SURVEY.md §8e), inside the timed region")
    return p.parse_args()


def cpu_baseline(model, period: int, target_s: float):
    """fp64 CPU oracle (oracle/oracle.c, 'port') on the host cores: bounded sample of the same
    workload (same scene, same synthetic inputs), one env per pthread task."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import binding
    from mujoco_ros2_simulation_amd import synth
    cores = max(1, min(16, os.cpu_count() or 1))
    # pilot: estimate env-step cost, then size the sample for ~target_s seconds
    n_pilot = cores
    steps = 100
    q0 = synth.initial_qpos(model, np.arange(n_pilot))
    tab = synth.ctrl_table(model, np.arange(n_pilot), steps // period + 1, period)
    secs, _, _ = binding.rollout(model, q0, tab, steps, period, cores)
    rate = n_pilot * steps / max(secs, 1e-6)
    n_envs = max(cores, int(round(rate * target_s / 500 / cores)) * cores)
    steps = 500
    q0 = synth.initial_qpos(model, np.arange(n_envs))
    tab = synth.ctrl_table(model, np.arange(n_envs), steps // period + 1, period)
    secs, _, _ = binding.rollout(model, q0, tab, steps, period, cores)
    return {"value": n_envs * steps / secs, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{n_envs} envs x {steps} steps of the same scene and synthetic inputs, fp64 oracle "
                      f"(oracle/oracle.c), {cores} pthreads, {secs:.1f} s"}


def measured_traffic(cfg: str, envs: int, period: int):
    """HBM bytes per launch of the config's dominant kernel from the committed rocprofv3 PMC summary of
    this same bench command (scripts/gpu_full.sh -> scripts/pmc_summary.py ->
    profiles/<round>/pmc_<cfg>.json); None when no summary exists for this workload."""
    default_envs = {"c3": 8192, "c4": 2048, "c5": 8192}
    if cfg not in default_envs or envs != default_envs[cfg] or period != 10:
        return None, None
    found = sorted(ROOT.glob(f"profiles/r*/pmc_{cfg}.json"))
    if not found:
        return None, None
    rec = json.loads(found[-1].read_text())
    return rec["traffic_bytes_per_launch"], str(found[-1].relative_to(ROOT))


def run_c4(args):
    """Config C4: scenes/mobile_base.xml, 2048 envs per GPU (16384 over 8), one bench
    step = one 10-step controller period; every --render-every physics steps (100: the reference's
    5 Hz camera rate at 500 Hz physics) a 640x480 depth frame of every env into HBM.  The roofline is
    the depth kernel's (HBM-bound: 1,228,800 B written per env-frame)."""
    import torch
    from mujoco_ros2_simulation_amd import shard, sim, synth
    rank, world, local = shard.init("nccl")
    torch.cuda.set_device(local)
    scene = ROOT / "scenes" / "mobile_base.xml"
    model = sim.Model.load(scene)
    n = args.envs if args.envs != 8192 else 2048
    ids = shard.env_ids(rank, n)
    P = args.warmup + args.steps
    d_table = torch.from_numpy(synth.ctrl_table(model, ids, P, args.period).astype(np.float32)).to(f"cuda:{local}")
    stream = torch.cuda.Stream(device=local)
    batch = sim.Batch(model, n, device=local)
    batch.set_stream(stream.cuda_stream)
    batch.set(sim.FIELD_QPOS, synth.initial_qpos(model, ids))
    W, H = int(model.cam_resolution[0, 0]), int(model.cam_resolution[0, 1])
    frames = torch.empty((n, H, W), dtype=torch.float32, device=f"cuda:{local}")
    every = max(1, args.render_every // args.period)
    torch.cuda.synchronize()
    step_ev, rend_ev = [], []

    def period(p, timed):
        batch.set_ctrl_device(d_table[p].data_ptr())
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else None
        if e: e[0].record(stream)
        batch.step(args.period)
        if e: e[1].record(stream); step_ev.append(e)
        if (p + 1) % every == 0:
            r = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else None
            if r: r[0].record(stream)
            batch.render_depth_device(0, 0, n, frames.data_ptr())
            if r: r[1].record(stream); rend_ev.append(r)

    with torch.cuda.stream(stream):
        for p in range(args.warmup):
            period(p, False)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        for k in range(args.steps):
            period(args.warmup + k, True)
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        t1 = time.perf_counter()
    step_ms = float(np.mean([a.elapsed_time(b) for a, b in step_ev]))
    rend_ms = float(np.mean([a.elapsed_time(b) for a, b in rend_ev])) if rend_ev else float("nan")
    elapsed, step_ms, rend_ms = shard.max_over_ranks([t1 - t0, step_ms, rend_ms], device=f"cuda:{local}")
    assert torch.isfinite(frames).all(), "non-finite depth"
    bytes_frame = n * W * H * 4
    achieved = bytes_frame / (rend_ms * 1e-3) / 1e9
    traffic, traffic_src = measured_traffic("c4", n, args.period)
    result = {
        "metric": "env-steps/sec (whole node), mobile base + 32-beam lidar + 640x480 depth camera (C4)",
        "value": world * n * args.steps * args.period / elapsed,
        "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (Philox4x32-10 seeded wheel-speed commands and initial states; SURVEY.md §8d)",
        "config": {"workload": "mobile_base (C4: free base + 2 wheels, 32-ray lidar, 640x480 depth)",
                   "envs_per_gpu": n, "global_envs": world * n, "physics_steps_per_bench_step": args.period,
                   "depth_every_physics_steps": every * args.period, "parallelism": f"env-sharded x{world}"},
        "depth_frames_per_s": world * n * len(rend_ev) / elapsed,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                     "frac": achieved / 8000.0, "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_unit": "bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)",
                     "kernel": "depth_kernel (one 640x480 frame of every env)", "kernel_ms": rend_ms,
                     "algorithmic_bytes_per_launch": bytes_frame, "step_kernel_ms": step_ms},
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    batch.close()
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    if args.config == "c4":
        return run_c4(args)
    if args.config == "c5":
        # C5: 65536 envs over 8 GPUs = 8192 per GPU, same loop as C3
        args.scene = str(ROOT / "scenes" / "arm_boxes.xml")
    import torch
    import torch.distributed as dist
    from mujoco_ros2_simulation_amd import build, roofline, shard, sim, synth

    rank, world, local = shard.init("nccl")   # RCCL over xGMI; only barrier and max-time reduce
    torch.cuda.set_device(local)
    if not sim.LIB_PATH.exists():
        if rank == 0:
            build.build_lib()
        if world > 1:
            dist.barrier()

    model = sim.Model.load(args.scene)
    n = args.envs
    env_ids = shard.env_ids(rank, n)
    P = args.warmup + args.steps
    table = synth.ctrl_table(model, env_ids, P, args.period).astype(np.float32)   # [P, n, nu]
    qpos0 = synth.initial_qpos(model, env_ids)

    stream = torch.cuda.Stream(device=local)
    batch = sim.Batch(model, n, device=local)
    batch.set_stream(stream.cuda_stream)
    batch.set(sim.FIELD_QPOS, qpos0)
    d_table = torch.from_numpy(table).to(f"cuda:{local}")
    gather = shard.ObsGather(n, [model.nq, model.nv], device=f"cuda:{local}") if args.gather and world > 1 else None
    torch.cuda.synchronize()

    def period(p: int, ev=None):
        batch.set_ctrl_device(d_table[p].data_ptr())
        if ev is not None:
            ev[0].record(stream)
        batch.step(args.period)
        if ev is not None:
            ev[1].record(stream)
        if gather is not None:
            # observations of this period into HBM buffers, then grouped sends to rank 0
            q, v = gather.start(p)
            batch.get_device(sim.FIELD_QPOS, q.data_ptr())
            batch.get_device(sim.FIELD_QVEL, v.data_ptr())
            gather.launch()

    with torch.cuda.stream(stream):
        for p in range(args.warmup):
            period(p)
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.steps)]
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for k in range(args.steps):
            period(args.warmup + k, events[k])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    elapsed, kern_ms = shard.max_over_ranks([elapsed, kern_ms], device=f"cuda:{local}")

    # sanity: states finite after the run (a diverged run would be invalid)
    q = batch.get(sim.FIELD_QPOS, 0, min(n, 64))
    assert np.all(np.isfinite(q)), "non-finite state after benchmark"

    env_steps = world * n * args.steps * args.period
    value = env_steps / elapsed
    detailed_flops = roofline.flops_per_env_step(model)
    flops, survey_bytes = roofline.SURVEY_PER_ENV_STEP.get(Path(args.scene).stem, (detailed_flops, None))
    bytes_ = roofline.bytes_per_env_step(model, args.period)
    achieved_tf = n * args.period * flops / (kern_ms * 1e-3) / 1e12
    cfg = {"arm7_lidar": "c3", "arm_boxes": "c5"}.get(Path(args.scene).stem, "")
    traffic, traffic_src = measured_traffic(cfg, n, args.period)
    result = {
        "metric": METRIC if args.config == "c3" else "env-steps/sec (whole node), contact-rich arm + 8 free boxes (C5)",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Philox4x32-10 seeded actions and initial states; SURVEY.md §8d)",
        "config": {
            "workload": (f"{Path(args.scene).stem} (C5: 7-DoF arm + 8 free boxes, PGS {model.iterations} iterations)"
                         if args.config == "c5" else
                         f"{Path(args.scene).stem} (C3: 7-DoF arm + {sum(1 for i in range(model.nsensor) if model.sensor_type[i] == sim.SENS_RANGEFINDER)}-ray lidar, PGS)"),
            "envs_per_gpu": n,
            "global_envs": world * n,
            "physics_steps_per_bench_step": args.period,
            "timestep": model.timestep,
            "parallelism": f"env-sharded x{world}",
            "obs_gather": "per period (qpos, qvel) of every env to rank 0, RCCL batch_isend_irecv" if gather else None,
        },
        "roofline": {
            "bound": "mfma",
            "achieved": achieved_tf,
            "peak": roofline.PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tf / roofline.PEAK_FP32_TFLOPS,
            "traffic": traffic,
            "traffic_unit": "bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": n * args.period * roofline.bytes_per_env_step(model, args.period),
            "kernel": "step_kernel<false> (fused 10-step launch)",
            "kernel_ms": kern_ms,
            "flops_per_env_step": flops,
            "flops_source": "SURVEY.md §8(d) per-unit figure x envs x steps per launch",
            "flops_per_env_step_structural": detailed_flops,
            "algorithmic_bytes_per_env_step": bytes_,
            "note": "VALU-bound fp32 path; peak is the fp32 vector rate (= fp32 MFMA rate on gfx950)",
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(model, args.period, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    batch.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
