"""GPU parity of the full implicit integrator (mj_implicit with the RNE velocity derivative;
oracle.c integrate / orc_bias_vel states the restatement and its KATs, step.hip integrate_implicit
runs it: two com_vel + rne passes per dof for the derivative, LU of every tree block).
Tolerance: |gpu - cpu| <= 1e-5 * max(|cpu|, 1) (north_star)."""
import numpy as np
import pytest

from conftest import ARM7, REF_SCENE
from mujoco_ros2_simulation_amd import sim, synth
from test_gpu_solvers import _reseeded
import binding

pytestmark = pytest.mark.gpu

RTOL = 1e-5
SCENES = ARM7.parent


def implicit_scene(path) -> "sim.Model":
    xml = path.read_text()
    if 'integrator="implicitfast"' in xml:
        xml = xml.replace('integrator="implicitfast"', 'integrator="implicit"')
    else:  # the reference scene: its <option> sits in the included robot file
        xml = xml.replace('<include file="test_robot.xml"/>', '<include file="test_robot.xml"/><option integrator="implicit"/>')
    m = sim.Model.from_string(xml, str(path.parent))
    assert m.integrator == 2
    return m


@pytest.mark.parametrize("group", [16, 32, 64])
def test_implicit_rollout_reference_scene(group, monkeypatch):
    """the reference's 2-DoF arm (planar, so Coriolis / centrifugal forces are the whole bias) under
    integrator="implicit", 64 envs of synthetic servo commands, 1000 steps, every group width"""
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = implicit_scene(REF_SCENE)
    n, steps, period = 64, 1000, 10
    envs = np.arange(n)
    q0 = synth.initial_qpos(model, envs)
    table = synth.ctrl_table(model, envs, steps // period + 1, period)
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, q0)
    for p in range(steps // period):
        b.set(sim.FIELD_CTRL, table[p])
        b.step(period)
    q, v = b.get(sim.FIELD_QPOS), b.get(sim.FIELD_QVEL)
    b.close()
    worst = 0.0
    for e in range(0, n, 7):
        d = binding.OracleData(model)
        d.qpos[:] = q0[e]
        for p in range(steps // period):
            d.ctrl[:] = table[p, e]
            d.step(period)
        scale_q, scale_v = np.maximum(np.abs(d.qpos), 1), np.maximum(np.abs(d.qvel), 1)
        worst = max(worst, np.max(np.abs(q[e] - d.qpos) / scale_q), np.max(np.abs(v[e] - d.qvel) / scale_v))
    print(f"G={group}: worst rel err after {steps} steps {worst:.2e}")
    assert worst <= RTOL


@pytest.mark.parametrize("scene, n", [("arm7_lidar", 32), ("arm_boxes", 8), ("mobile_base", 32)])
def test_reseeded_implicit(scene, n):
    """scenes under integrator="implicit": every step from the oracle's state, qpos / qvel within 1e-5
    (16-lane groups with a lidar, blocked mode with contacts -- the derivative per tree block --, and
    a free-floating base whose gyroscopic terms the derivative carries)"""
    model = implicit_scene(SCENES / f"{scene}.xml")
    wq, wv, ncon, flips, unexplained = _reseeded(model, n, 40)
    print(f"{scene} implicit: worst per-step rel err qpos {wq:.2e} qvel {wv:.2e}; flips {flips}")
    assert flips <= max(1, 0.01 * n * 40)
    assert not unexplained, unexplained[:5]
    assert wq <= RTOL and wv <= RTOL
