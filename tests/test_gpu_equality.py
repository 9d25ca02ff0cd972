"""GPU parity of equality constraints (MJCF <equality>: connect, weld, joint; mjModel eq_*, rows of
mj_instantiateEquality restated in oracle.c equality_rows): per-step re-seeded parity within 1e-5
under PGS and Newton, on 16-lane groups and in blocked mode (G = 64), and a long rollout of a closed
chain that only the constraint holds together."""
import numpy as np
import pytest

from mujoco_ros2_simulation_amd import sim, synth
import binding

pytestmark = pytest.mark.gpu

EQ_SCENE = """<mujoco><option timestep="0.002" solver="{solver}" iterations="{it}"/><worldbody>
<geom name="floor" type="plane" size="0 0 1"/>
<body name="l1" pos="0 0 0.6"><joint name="h1" axis="0 1 0" damping="0.05"/><geom type="capsule" size="0.02" fromto="0 0 0 0.3 0 0"/>
  <body name="l2" pos="0.3 0 0"><joint name="h2" axis="0 1 0"/><geom type="capsule" size="0.02" fromto="0 0 0 0 0 -0.3"/></body></body>
<body name="l3" pos="0.6 0 0.6"><joint name="h3" axis="0 1 0"/><geom type="capsule" size="0.02" fromto="0 0 0 -0.3 0 -0.3"/></body>
<body name="box" pos="-0.4 0.3 0.5" euler="10 0 20"><freejoint/><geom type="box" size="0.05 0.04 0.03"/></body>
<body name="ball" pos="-0.4 0.3 0.35"><freejoint/><geom type="sphere" size="0.04"/></body>
<body name="w1" pos="0.3 -0.4 0.3"><joint name="s1" type="slide" axis="1 0 0"/><geom type="box" size="0.03 0.03 0.03"/></body>
<body name="w2" pos="0.3 -0.6 0.3"><joint name="s2" type="slide" axis="1 0 0"/><geom type="box" size="0.03 0.03 0.03"/></body>
</worldbody>
<equality><connect body1="l2" body2="l3" anchor="0 0 -0.3"/><weld body1="ball" body2="box"/>
  <joint joint1="s1" joint2="s2" polycoef="0 -1 0.5 0 0"/></equality>
<actuator><motor joint="h1" gear="5"/><motor joint="s2" gear="2"/></actuator></mujoco>"""


def scene(solver):
    it = {"PGS": "50", "Newton": "100"}[solver]
    return sim.Model.from_string(EQ_SCENE.format(solver=solver, it=it))


def test_equality_model():
    m = scene("PGS")
    assert m.neq == 3 and list(m.eq_type) == [sim.EQ_CONNECT, sim.EQ_WELD, sim.EQ_JOINT]
    d = binding.OracleData(m)
    d.forward()
    assert d.nefc >= 3 + 6 + 1


@pytest.mark.parametrize("solver", ["PGS", "Newton"])
@pytest.mark.parametrize("group", [16, 64])
def test_reseeded_equality(solver, group, monkeypatch):
    from test_gpu_solvers import _reseeded
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = scene(solver)
    wq, wv, ncon, flips, unexplained = _reseeded(model, 8, 60, settle=30)
    print(f"equality scene {solver} G={group}: worst per-step rel err qpos {wq:.2e} qvel {wv:.2e}; flips {flips}")
    assert not unexplained, unexplained[:5]
    assert wq <= 1e-5 and wv <= 1e-5


def test_closed_chain_rollout():
    """the four-bar (two links on hinges closed by a connect) under the motor for 1000 steps: the
    connect's anchor points stay together on the device (within the soft constraint's own sag, as
    the oracle's), and qpos follows the oracle within the scene's fp32 sensitivity"""
    # the chain's capsules do not collide here: a link grazing the floor is a contact threshold event
    # (present on one side only for a step), after which the chaotic swing separates the two rollouts
    # far beyond the rounding sensitivity measured below
    model = sim.Model.from_string(EQ_SCENE.format(solver="PGS", it="50").replace(
        '<geom type="capsule"', '<geom type="capsule" contype="0" conaffinity="0"'))
    n, steps = 4, 1000
    q0 = synth.initial_qpos(model, np.arange(n))
    tab = synth.ctrl_table(model, np.arange(n), steps // 10 + 1, 10)
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, q0)
    for p in range(steps // 10):
        b.set(sim.FIELD_CTRL, tab[p])
        b.step(10)
    q = b.get(sim.FIELD_QPOS)
    b.close()
    for e in range(n):
        outs = []
        for rnd in (False, True):
            d = binding.OracleData(model)
            d.qpos[:] = q0[e]
            for p in range(steps // 10):
                d.ctrl[:] = tab[p, e]
                for _ in range(10):
                    d.step()
                    if rnd:
                        d.qpos[:] = d.qpos.astype(np.float32)
                        d.qvel[:] = d.qvel.astype(np.float32)
            outs.append(d.qpos.copy())
        ref, ref32 = outs
        # the hinge chain's coordinates (h1, h2, h3): chaotic contact-free dynamics stay smooth here
        err = np.max(np.abs(q[e, :3] - ref[:3]))
        sens = np.max(np.abs(ref32[:3] - ref[:3]))
        assert err <= 10 * sens + 1e-4, (e, err, sens)
