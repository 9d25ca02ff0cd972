"""GPU parity of the RK4 integrator (mj_RungeKutta(m, d, 4); oracle.c rk4 states the restatement,
step.hip rk4_stage / rk4_final run the three extra stages around the step loop's forward).
Tolerance: |gpu - cpu| <= 1e-5 * max(|cpu|, 1) (north_star)."""
import numpy as np
import pytest

from conftest import ARM7
from mujoco_ros2_simulation_amd import sim
from test_gpu_solvers import _reseeded, _rel
from test_oracle_kat import SERVO
import binding

pytestmark = pytest.mark.gpu

RTOL = 1e-5
SCENES = ARM7.parent


def rk4_scene(name: str, solver: str | None = None) -> "sim.Model":
    path = SCENES / f"{name}.xml"
    xml = path.read_text().replace('integrator="implicitfast"', 'integrator="RK4"')
    if solver:
        xml = xml.replace('solver="PGS"', f'solver="{solver}"')
    assert 'integrator="RK4"' in xml
    return sim.Model.from_string(xml, str(path.parent))


def test_servo_rk4_rollout():
    """the damped servo of the oracle KAT, 64 envs with different set points, 1000 steps"""
    I, b, kp, kv = 0.5, 0.3, 40.0, 2.0
    m = sim.Model.from_string(SERVO.format(integ="RK4", b=b, I=I, kp=kp, kv=kv))
    n = 64
    ctrl = np.linspace(-1.0, 1.0, n)[:, None]
    bt = sim.Batch(m, n)
    bt.set(sim.FIELD_CTRL, ctrl)
    bt.step(1000)
    q, v = bt.get(sim.FIELD_QPOS), bt.get(sim.FIELD_QVEL)
    for e in (0, 17, 63):
        d = binding.OracleData(m)
        d.ctrl[:] = ctrl[e]
        d.step(1000)
        assert _rel(q[e], d.qpos) <= RTOL and _rel(v[e], d.qvel) <= RTOL


@pytest.mark.parametrize("scene, solver, n", [("arm7_lidar", None, 32), ("arm_boxes", None, 8),
                                             ("arm7_lidar", "Newton", 32)])
def test_reseeded_rk4(scene, solver, n):
    """scenes under RK4: every step from the oracle's state, qpos / qvel within 1e-5 (16-lane groups
    with PGS, blocked mode with contacts, and the Newton kernel).  (The mobile base is not used: its
    stiff wheel velocity servos are unstable under explicit RK4 at its 2 ms step -- the oracle itself
    reaches |qvel| ~ 1e9 and auto-resets, which is the integrator's behaviour, not a parity case.)"""
    model = rk4_scene(scene, solver)
    # (contacts of an RK4 step are those of its last stage's forward, not of the start state that
    # flips.explain_flip perturbs, so only the flip count is bounded here)
    wq, wv, ncon, flips, _ = _reseeded(model, n, 60)
    print(f"{scene} RK4 {solver or 'PGS'}: worst per-step rel err qpos {wq:.2e} qvel {wv:.2e}; flips {flips}")
    assert flips <= 0.01 * n * 60
    assert wq <= RTOL and wv <= RTOL
