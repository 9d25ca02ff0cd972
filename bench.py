#!/usr/bin/env python3
"""Benchmark: batched mj_step on MI355X (BASELINE.json metric "env-steps/sec (whole node),
7-DoF arm+lidar scene").

Workload (BASELINE.json configs[2]): scenes/arm7_lidar.xml — 7-DoF arm,
360-beam rangefinder lidar, PGS — 8192 envs per GPU (weak scaling: every rank owns its own 8192
envs, global env ids rank*8192 + i, no data-path collective).  One bench "step" = one controller
period = 10 physics steps (mj_step) of every env with the period's synthetic action held (the
reference's 500 Hz physics / 50 Hz controller ratio), i.e. one fused kernel launch.  Inputs (the
whole synthetic action table) are resident in HBM before timing starts.  With N > 1 ranks every
period ends with the observation gather of SURVEY.md §8e (each rank's (qpos, qvel) to rank 0 over
RCCL point-to-point), inside the timed region.

Other configs (`--config`): c2 = the reference's 2-DoF scene (Newton, its default solver), 4096
envs, sensors disabled; c4 = mobile base + 32-beam lidar + 640x480 depth camera, 2048 envs per GPU;
c5 = arm + 8 free boxes, PGS 50 iterations, 8192 envs per GPU.

Prints ONE JSON line on rank 0.  Launch: `python bench.py` (1 GPU); `python bench.py --gpus N`
spawns N ranks itself (one process per GPU, before any GPU call); under torchrun
(`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`) each rank runs directly.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "env-steps/sec (whole node), 7-DoF arm+lidar scene at 1/2/4/8 MI355X"
REF_SCENE = ROOT / "tests" / "golden" / "ref_scenes" / "scene.xml"   # reference test scene (data fixture)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200, help="timed controller periods")
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--period", type=int, default=10, help="physics steps per controller period")
    p.add_argument("--envs", type=int, default=0, help="envs per GPU (0: the config's default)")
    p.add_argument("--scene", default=None, help="override the config's scene")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    p.add_argument("--config", choices=["c1", "c2", "c3", "c3m", "c4", "c5"], default="c3",
                   help="c3: the BASELINE metric (default); c1: the reference scene, 1 env, through the plugin host "
                        "(MujocoSystemInterface, headless), paced and unpaced; "
                        "c2: reference 2-DoF scene, 4096 envs, sensors off; "
                        "c4: mobile base + lidar + 640x480 depth camera; c5: contact-rich arm + 8 free boxes; "
                        "c3m: C3 with mesh link shells and a 6912-triangle statue + a 640x480 camera (ray hierarchy)")
    p.add_argument("--c1-seconds", type=float, default=3.0, help="C1: wall seconds of the paced measurement")
    p.add_argument("--render-every", type=int, default=100, help="C4: physics steps between depth frames")
    p.add_argument("--render-sync", action="store_true",
                   help="C4: render each frame on the batch stream between steps instead of the camera "
                        "pipeline (pose snapshot, render concurrently with the following steps)")
    p.add_argument("--solver", choices=["PGS", "CG", "Newton"], default=None,
                   help="override the scene's <option solver> (e.g. c5 under MuJoCo's default Newton)")
    p.add_argument("--no-gather", action="store_true",
                   help="N>1: skip the end-of-period observation gather (on by default when N > 1)")
    return p.parse_args()


# ------------------------------------------------------------------------------------------------ CPU baseline
def host_cores():
    """(cores usable by this process, visible CPUs, model name): the affinity mask bounded by the
    cgroup CPU quota (a container may see every CPU of the host but be granted fewer)."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    cores = visible if quota is None else max(1, min(visible, math.floor(quota)))
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return min(cores, 256), visible, quota, model


def cpu_baseline(model, period: int, target_s: float):
    """fp64 CPU oracle (oracle/oracle.c, 'port') on every host core this process may use, one pinned
    pthread per core: bounded sample of the same workload (same scene, same synthetic inputs)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import binding
    from mujoco_ros2_simulation_amd import synth
    cores, visible, quota, cpu_model = host_cores()
    n_pilot = cores
    steps = 100
    q0 = synth.initial_qpos(model, np.arange(n_pilot))
    tab = synth.ctrl_table(model, np.arange(n_pilot), steps // period + 1, period)
    secs, _, _ = binding.rollout(model, q0, tab, steps, period, cores)
    rate = n_pilot * steps / max(secs, 1e-6)
    steps = 500
    n_envs = max(cores, int(round(rate * target_s / steps / cores)) * cores)
    q0 = synth.initial_qpos(model, np.arange(n_envs))
    tab = synth.ctrl_table(model, np.arange(n_envs), steps // period + 1, period)
    secs, _, _ = binding.rollout(model, q0, tab, steps, period, cores)
    return {"value": n_envs * steps / secs, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model, "cpus_visible": visible, "cpu_quota": quota, "pinned": cores <= visible,
            "sample": f"{n_envs} envs x {steps} steps of the same scene and synthetic inputs, fp64 CPU restatement "
                      f"(oracle/oracle.c, not upstream MuJoCo), {cores} pinned pthreads on {cpu_model}, {secs:.1f} s"}


# ------------------------------------------------------------------------------------------------ evidence
def variant_key(cfg: str, solver: str | None, scene: str | None) -> str:
    """file key of one bench command's counter summaries: the config, plus the solver and scene when
    they override the config's own (e.g. c5_newton, c3_arm7_lidar1080), so a bench line never
    carries the counters of a different kernel run (scripts/gpu_evidence.sh collects them per key)"""
    key = cfg
    if solver:
        key += "_" + solver.lower()
    if scene:
        key += "_" + Path(scene).stem
    return key


def committed(kind: str, cfg: str, envs: int, period: int, key: str | None = None):
    """newest committed rocprofv3 PMC summary `profiles/r*/<kind>_<key>.json` of this same bench
    command (scripts/gpu_evidence.sh -> scripts/pmc_summary.py); None for other workload sizes or
    when no summary of exactly this variant (config + solver + scene) was collected"""
    default_envs = {"c2": 4096, "c3": 8192, "c3m": 8192, "c4": 2048, "c5": 8192}
    if cfg not in default_envs or envs != default_envs[cfg] or period != 10:
        return None, None
    found = sorted(ROOT.glob(f"profiles/r*/{kind}_{key or cfg}.json"))
    if not found:
        return None, None
    return json.loads(found[-1].read_text()), str(found[-1].relative_to(ROOT))


def ref_scene_xml(sensors: bool) -> tuple[str, str]:
    """C2 scene: the reference's resources/scene.xml (= test/test_resources/scene.xml with the 2-DoF
    robot included), optionally with <flag sensor="disable"/> (no sensors)."""
    xml = REF_SCENE.read_text()
    if not sensors:
        i = xml.index(">", xml.index("<mujoco")) + 1
        xml = xml[:i] + '\n  <option><flag sensor="disable"/></option>' + xml[i:]
    return xml, str(REF_SCENE.parent)


def with_solver(xml: str, solver: str) -> str:
    """the scene with <option solver=...> set (inserted when the scene has no <option>)"""
    import re
    m = re.search(r"<option\b[^>]*?/?>", xml)
    if m is None:
        i = xml.index(">", xml.index("<mujoco")) + 1
        return xml[:i] + f'\n  <option solver="{solver}"/>' + xml[i:]
    tag = re.sub(r'\ssolver="[^"]*"', "", m.group(0))
    tag = tag.replace("<option", f'<option solver="{solver}"', 1)
    return xml[:m.start()] + tag + xml[m.end():]


# ------------------------------------------------------------------------------------------------ C1
def run_c1(args):
    """BASELINE.json configs[0]: the reference's own scene, 1 env, driven through
    the plugin host exactly as the controller manager drives MujocoSystemInterface (headless=true,
    test/test_resources/test_robot.urdf with its <ros2_control> block; libmrs_plugin.so over the GPU
    batch, no CPU path).  Two rates:
    * paced: the physics thread (PhysicsLoop, reference src/mujoco_system_interface.cpp:1629-1780)
      with the URDF's sim_speed_factor 3.0 while a 50 Hz controller loop calls write()/read() -- sim
      steps per wall second, 1500 by construction of the pacing;
    * unpaced (the reported value): physics_thread=false, controller cycles back to back, each one
      write() + 10 physics steps (one fused launch) + read() -- the plumbing ceiling of one env."""
    import tempfile
    from mujoco_ros2_simulation_amd import plugin, sim
    gold = ROOT / "tests" / "golden"
    share = Path(tempfile.mkdtemp(prefix="mrs_c1_")) / "mujoco_ros2_control"
    share.mkdir()
    os.symlink(gold / "ref_scenes", share / "test_resources")
    os.symlink(gold / "ref_config", share / "config")
    urdf = gold / "ref_config" / "test_robot.urdf"

    def system(**params):
        s = plugin.System(urdf, {"use_pid": "false", "headless": "true"}, {"mujoco_ros2_control": str(share)})
        for k, v in params.items():
            s.set_param(k, v)
        if s.on_init() != plugin.SUCCESS:
            raise RuntimeError("on_init failed")
        s.on_activate()
        s.set_command("joint1/position", 0.5)
        s.set_command("joint2/position", -0.5)
        return s

    ctrl_period = 1.0 / 50  # test/config/controllers.yaml:3
    # paced: the physics thread against the wall clock
    s = system()
    h = s.get_model()["timestep"]
    speed = float(s.param("sim_speed_factor"))
    end = time.monotonic() + 0.5
    while time.monotonic() < end:
        s.write(ctrl_period); time.sleep(ctrl_period); s.read()
    t0w, t0s = time.monotonic(), s.sim_time
    end = t0w + args.c1_seconds
    while time.monotonic() < end:
        s.write(ctrl_period); time.sleep(ctrl_period); s.read()
    paced = (s.sim_time - t0s) / h / (time.monotonic() - t0w)
    s.close()
    # unpaced: synchronous controller cycles
    s = system(physics_thread="false")
    bh = s.batch_handle()
    sim.lib().mrs_batch_set_timing(bh, 3)  # (the kernel time of each cycle below)
    for _ in range(args.warmup):
        s.cycle(ctrl_period, args.period)
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s.cycle(ctrl_period, args.period)
        kms.append(sim.lib().mrs_batch_last_kernel_ms(bh, 0))
    elapsed = time.perf_counter() - t0
    q = np.array([s.state("joint1/position"), s.state("joint2/position")])
    assert np.all(np.isfinite(q))
    # single physics steps, one per call (each a launch + synchronous state copy)
    n1 = max(50, args.steps)
    t1 = time.perf_counter()
    for _ in range(n1):
        s.step(1)
    single = n1 / (time.perf_counter() - t1)
    s.close()
    value = args.steps * args.period / elapsed
    kernel_ms = float(np.mean(kms))
    result = {
        "metric": "env-steps/sec, reference scene, 1 env through MujocoSystemInterface headless (C1)",
        "value": value, "unit": "env-steps/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "the reference's test robot (test/test_resources/test_robot.urdf + scene.xml), commands [0.5, -0.5]",
        "config": {"workload": "C1: resources/scene.xml (2-DoF test robot), 1 env, plugin host, headless",
                   "envs_per_gpu": 1, "physics_steps_per_bench_step": args.period, "timestep": h,
                   "bench_step": "one controller cycle: write() + 10 physics steps (one launch) + read()",
                   "parallelism": "none (1 env)"},
        "paced_steps_per_s": paced, "paced_expected": speed / h, "sim_speed_factor": speed,
        "unpaced_single_step_per_s": single,
        "roofline": {"bound": "latency", "achieved": None, "peak": None, "unit": None, "frac": None,
                     "traffic": None, "kernel": "step_kernel<16, false, true> (10-step launch of 1 env; Newton kernel)",
                     "kernel_ms": kernel_ms,
                     "note": "one env occupies one 16-lane group of one wave: a launch- and copy-latency "
                             "measurement, not a roofline one; host overhead per cycle = ms_per_step - kernel_ms"},
    }
    if not args.no_cpu_baseline:
        sys.path.insert(0, str(ROOT / "oracle"))
        import binding
        cores, visible, quota, cpu_model = host_cores()
        m = sim.Model.load(gold / "ref_scenes" / "scene.xml")
        d = binding.OracleData(m)
        d.ctrl[:] = [0.5, -0.5]
        steps, t2 = 0, time.perf_counter()
        while time.perf_counter() - t2 < min(args.cpu_seconds, 5.0):
            d.step(1000)
            steps += 1000
        secs = time.perf_counter() - t2
        result["cpu_baseline"] = {"value": steps / secs, "unit": "env-steps/s", "cores": 1, "kind": "port",
                                  "cpu_model": cpu_model,
                                  "sample": f"1 env x {steps} mj_step of the same scene, fp64 CPU restatement "
                                            f"(oracle/oracle.c, not upstream MuJoCo), 1 thread, {secs:.1f} s"}
    print(json.dumps(result), flush=True)


# ------------------------------------------------------------------------------------------------ run
def main():
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "0"))
    if args.gpus > 1 and world_env == 0:
        # one process per GPU, started before anything here touches the GPU
        from mujoco_ros2_simulation_amd import shard
        sys.exit(shard.spawn(args.gpus, [str(Path(__file__).resolve())] + sys.argv[1:]))
    if world_env and world_env != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} does not match WORLD_SIZE={world_env}")
    if args.config == "c1":
        if args.gpus != 1:
            sys.exit("bench.py: --config c1 is the single-env plumbing case (1 GPU)")
        return run_c1(args)

    import torch
    import torch.distributed as dist
    from mujoco_ros2_simulation_amd import roofline, shard, sim, synth

    rank, world, local = shard.init("nccl")   # RCCL over xGMI: barrier, max-time reduce, obs gather
    torch.cuda.set_device(local)
    dev = f"cuda:{local}"
    cfg = args.config
    vkey = variant_key(cfg, args.solver, args.scene)
    if args.scene:
        path = Path(args.scene)
        xml, base = path.read_text(), str(path.parent)
        scene_name = path.stem
    elif cfg == "c2":
        xml, base = ref_scene_xml(sensors=False)
        scene_name = "scene"
    else:
        scene_name = {"c3": "arm7_lidar", "c3m": "arm7_mesh", "c4": "mobile_base", "c5": "arm_boxes"}[cfg]
        path = ROOT / "scenes" / f"{scene_name}.xml"
        xml, base = path.read_text(), str(path.parent)
    if args.solver:
        xml = with_solver(xml, args.solver)
    model = sim.Model.from_string(xml, base)
    n = args.envs or {"c2": 4096, "c3": 8192, "c3m": 8192, "c4": 2048, "c5": 8192}[cfg]
    env_ids = shard.env_ids(rank, n)
    P = args.warmup + args.steps
    d_table = torch.from_numpy(synth.ctrl_table(model, env_ids, P, args.period).astype(np.float32)).to(dev)

    stream = torch.cuda.Stream(device=local)
    batch = sim.Batch(model, n, device=local)
    batch.set_stream(stream.cuda_stream)
    # step launches are bracketed by this script's own HIP events (below), not by the batch's (a
    # second pair around every launch cost ~10 us, mrs_batch_set_timing); frames are timed by the batch
    batch.set_timing(2)
    batch.set(sim.FIELD_QPOS, synth.initial_qpos(model, env_ids))
    gather = None
    if world > 1 and not args.no_gather:
        gather = shard.ObsGather(n, [model.nq, model.nv], device=dev)
    render = cfg in ("c4", "c3m")
    if render:
        W, H = int(model.cam_resolution[0, 0]), int(model.cam_resolution[0, 1])
        frames = torch.empty((n, H, W), dtype=torch.float32, device=dev)
        every = max(1, args.render_every // args.period)
    torch.cuda.synchronize()
    step_ev, rend_ev = [], []
    rend_async, rend_async_ms = [False], []

    def period(p: int, timed: bool):
        # the period's actions, resident in HBM, bound as the launch's ctrl source (zero-copy
        # mrs_batch_bind_ctrl_device: the kernel loads them at launch start; no copy op between
        # launches)
        batch.bind_ctrl_device(d_table[p].data_ptr())
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else None
        if e:
            e[0].record(stream)
        batch.step(args.period)
        if e:
            e[1].record(stream)
            step_ev.append(e)
        if render and (p + 1) % every == 0:
            if args.render_sync:
                r = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else None
                if r:
                    r[0].record(stream)
                batch.render_depth_device(0, 0, n, frames.data_ptr())
                if r:
                    r[1].record(stream)
                    rend_ev.append(r)
            else:
                # the reference's camera thread: snapshot now, render while the next periods step.
                # The previous frame's kernel time (HIP events on the render stream) is read first.
                if rend_async[0]:
                    rend_async_ms.append(batch.last_kernel_ms(1))
                batch.render_async(0, 0, n, frames.data_ptr())
                rend_async[0] = timed
        if gather is not None:
            # this period's observations into HBM buffers, then grouped sends to rank 0
            q, v = gather.start(p)
            batch.get_device(sim.FIELD_QPOS, q.data_ptr())
            batch.get_device(sim.FIELD_QVEL, v.data_ptr())
            gather.launch()

    with torch.cuda.stream(stream):
        for p in range(args.warmup):
            period(p, False)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for k in range(args.steps):
            period(args.warmup + k, True)
        if gather is not None:
            gather.gathered(args.warmup + args.steps - 1)
        if render and not args.render_sync:
            batch.render_wait()   # the last frame is part of the timed work
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
    batch.sync()
    step_ms = float(np.mean([a.elapsed_time(b) for a, b in step_ev]))
    if rend_async[0]:
        rend_async_ms.append(batch.last_kernel_ms(1))
    rend_list = rend_async_ms if not args.render_sync else [a.elapsed_time(b) for a, b in rend_ev]
    rend_ms = float(np.mean(rend_list)) if rend_list else float("nan")
    elapsed, step_ms, rend_ms = shard.max_over_ranks([t1 - t0, step_ms, rend_ms], device=dev)

    # sanity: states finite after the run (a diverged run would be invalid)
    q = batch.get(sim.FIELD_QPOS, 0, min(n, 64))
    assert np.all(np.isfinite(q)), "non-finite state after benchmark"
    if render:
        assert torch.isfinite(frames).all(), "non-finite depth"

    value = world * n * args.steps * args.period / elapsed
    solver = {0: "PGS", 1: "CG", 2: "Newton"}[model.solver]
    nrf = sum(1 for i in range(model.nsensor) if model.sensor_type[i] == sim.SENS_RANGEFINDER)
    workload = {
        "c2": f"reference 2-DoF scene (C2: resources/scene.xml, sensors disabled, {solver})",
        "c3": f"{scene_name} (C3: 7-DoF arm + {nrf}-ray lidar, {solver})",
        "c4": f"{scene_name} (C4: free base + 2 wheels, {nrf}-ray lidar, 640x480 depth, {solver})",
        "c3m": f"{scene_name} (C3 with mesh link shells + a 6912-triangle statue, {nrf}-ray lidar, "
               f"640x480 depth, {solver})",
        "c5": f"{scene_name} (C5: 7-DoF arm + 8 free boxes, {solver} {model.iterations} iterations)",
    }[cfg]
    metric = {
        "c2": "env-steps/sec (whole node), reference 2-DoF scene, no sensors (C2)",
        "c3": METRIC,
        "c4": "env-steps/sec (whole node), mobile base + 32-beam lidar + 640x480 depth camera (C4)",
        "c5": "env-steps/sec (whole node), contact-rich arm + 8 free boxes (C5)",
        "c3m": "env-steps/sec (whole node), mesh robot: C3 + mesh shells, statue, 640x480 depth (C3m)",
    }[cfg]
    config = {"workload": workload, "envs_per_gpu": n, "global_envs": world * n,
              "physics_steps_per_bench_step": args.period, "timestep": model.timestep,
              "parallelism": f"env-sharded x{world}",
              "obs_gather": ("per period (qpos, qvel) of every env to rank 0, RCCL batch_isend_irecv"
                             if gather is not None else None)}
    traffic_rec, traffic_src = committed("pmc", cfg, n, args.period, vkey)
    sq_rec, sq_src = committed("sq", cfg, n, args.period, vkey)
    if render:
        config["depth_every_physics_steps"] = every * args.period
        config["camera_pipeline"] = ("frames rendered on the batch stream between steps" if args.render_sync else
                                     "pose snapshot on the batch stream, frame rendered on a second HIP stream "
                                     "concurrently with the following steps (the reference's rendering thread)")
        bytes_frame = n * W * H * 4
        achieved = bytes_frame / (rend_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": roofline.PEAK_HBM_GBS, "unit": "GB/s",
                "frac": achieved / roofline.PEAK_HBM_GBS,
                "traffic": traffic_rec["traffic_bytes_per_launch"] if traffic_rec else None,
                "traffic_source": traffic_src, "traffic_unit": "bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)",
                "kernel": (("depth_kernel_mesh (triangle-binned" if model.nmesh > 0 else "depth_kernel_v2 (tiled") +
                           f", one {W}x{H} frame of every env)"), "kernel_ms": rend_ms,
                "algorithmic_bytes_per_launch": bytes_frame, "step_kernel_ms": step_ms}
    else:
        detailed_flops = roofline.flops_per_env_step(model)
        flops, _ = roofline.SURVEY_PER_ENV_STEP.get(scene_name, (detailed_flops, None))
        achieved_tf = n * args.period * flops / (step_ms * 1e-3) / 1e12
        roof = {"bound": "valu", "achieved": achieved_tf, "peak": roofline.PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved_tf / roofline.PEAK_FP32_TFLOPS,
                "traffic": traffic_rec["traffic_bytes_per_launch"] if traffic_rec else None,
                "traffic_unit": "bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)", "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": n * args.period * roofline.bytes_per_env_step(model, args.period),
                "kernel": "step_kernel<G, false, *> (fused 10-step launch)", "kernel_ms": step_ms,
                "flops_per_env_step": flops,
                "flops_source": "SURVEY.md §8(d) per-unit figure x envs x steps per launch",
                "flops_per_env_step_structural": detailed_flops,
                "algorithmic_bytes_per_env_step": roofline.bytes_per_env_step(model, args.period),
                "note": "fp32 vector-ALU bound path (no GEMM-shaped work at these sizes); peak = fp32 VALU rate"}
    fl_rec, fl_src = committed("flops", cfg, n, args.period, vkey)
    if not render:
        roof["frac_model"] = roof["frac"]
        if fl_rec:
            # executed fp32 VALU work of the same kernel (rocprofv3 SQ_INSTS_VALU_*_F32 /
            # SQ_INSTS_VALU_FLOPS_FP32 of this bench command, scripts/flops_summary.py), timed here
            fe = fl_rec["flops_executed_per_env_step"]
            roof["flops_executed_per_env_step"] = fe
            roof["frac_executed"] = n * args.period * fe / (step_ms * 1e-3) / 1e12 / roofline.PEAK_FP32_TFLOPS
            roof["flops_executed_source"] = fl_src
            roof["flops_executed_note"] = ("fp32 VALU instructions x 64 lanes (2 per FMA) of this kernel, "
                                           "rocprofv3 SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F32: an upper bound "
                                           "(idle lanes of a 16-lane group count)")
    if sq_rec:
        # measured from SQ counters of the same command (rocprofv3 --pmc, scripts/sq_summary.py)
        roof["valu_measured"] = {k: sq_rec[k] for k in ("valu_issue_frac", "valu_tflops_upper", "valu_frac_upper",
                                                        "wait_frac", "waves_per_simd") if k in sq_rec}
        roof["valu_measured"]["source"] = sq_src
    result = {
        "metric": metric, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (Philox4x32-10 seeded actions and initial states; SURVEY.md §8d)",
        "config": config, "roofline": roof,
    }
    if render:
        result["depth_frames_per_s"] = world * n * len(rend_list) / elapsed
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(model, args.period, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    batch.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
