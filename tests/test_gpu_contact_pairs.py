"""GPU parity of explicit contact pairs and excluded body pairs (MJCF <contact><pair> / <exclude>,
mjModel pair_* / exclude_signature): an explicit pair collides geoms that
contype/conaffinity keep apart, with its own friction / solref; an excluded body pair never collides;
the contact list (geom1, geom2) is bit-exact against the oracle and the per-step re-seeded state
within 1e-5."""
import numpy as np
import pytest

from mujoco_ros2_simulation_amd import sim, synth
import binding

pytestmark = pytest.mark.gpu

PAIR_SCENE = """<mujoco><option timestep="0.002" solver="PGS" iterations="50"/>
<default><pair solref="0.01 1"/></default>
<worldbody><geom name="floor" type="plane" size="0 0 1"/>
<body name="a" pos="0 0 0.1" euler="5 3 0"><freejoint/><geom name="ga" type="box" size="0.1 0.08 0.06" contype="0" conaffinity="0"/></body>
<body name="b" pos="0.35 0 0.1"><freejoint/><geom name="gb" type="sphere" size="0.1"/></body>
<body name="c" pos="0.37 0.02 0.32"><freejoint/><geom name="gc" type="sphere" size="0.1"/></body>
<body name="d" pos="-0.3 0.1 0.12" euler="0 80 0"><freejoint/><geom name="gd" type="capsule" size="0.04 0.1"/></body>
</worldbody>
<contact><pair geom1="ga" geom2="floor" friction="0.5 0.5 0.01 0.001 0.001"/>
  <pair geom1="gd" geom2="floor" condim="1"/><exclude body1="b" body2="c"/></contact>
</mujoco>"""


def test_pair_contacts_match_oracle():
    model = sim.Model.from_string(PAIR_SCENE)
    assert model.nexpair == 2 and model.nexclude == 1
    n = 8
    q0 = synth.initial_qpos(model, np.arange(n))
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, q0)
    b.step(60)
    q = b.get(sim.FIELD_QPOS)
    b.forward()
    seen = set()
    for e in range(n):
        g, dist, pos, frame = b.contacts(e)
        d = binding.OracleData(model)
        d.qpos[:] = q[e]
        d.forward()
        gr, dr, pr, fr = d.contacts()
        assert np.array_equal(g, gr), (e, g.tolist(), gr.tolist())
        np.testing.assert_allclose(dist, dr, atol=1e-5)
        seen |= {tuple(x) for x in g.tolist()}
    assert (0, 1) in seen and (0, 4) in seen      # explicit pairs: box (contype 0) and capsule on the floor
    assert (2, 3) not in seen and (3, 2) not in seen  # excluded: the stacked spheres fall through each other


def test_reseeded_pairs():
    from test_gpu_solvers import _reseeded
    model = sim.Model.from_string(PAIR_SCENE)
    wq, wv, ncon, flips, unexplained = _reseeded(model, 8, 100, settle=40)
    print(f"pair scene: worst per-step rel err qpos {wq:.2e} qvel {wv:.2e}; contacts {ncon.mean():.2f}; flips {flips}")
    assert ncon.max() > 0
    assert not unexplained, unexplained[:5]
    assert wq <= 1e-5 and wv <= 1e-5


# one body, two geoms: only the foot has an explicit pair with the floor.  The merge skips only that
# geom pair, so the body's second geom (a knee sphere, lower than the foot) still gets its dynamic
# floor contact (mj_collision merge [upstream; verify])
TWO_GEOM_BODY = """<mujoco><option timestep="0.002" solver="PGS" iterations="50"/>
<worldbody><geom name="floor" type="plane" size="0 0 1"/>
<body name="leg" pos="0 0 0.12"><freejoint/>
  <geom name="foot" type="box" size="0.1 0.05 0.03" pos="0.2 0 0"/>
  <geom name="knee" type="sphere" size="0.06" pos="-0.2 0 -0.05"/></body>
</worldbody>
<contact><pair geom1="foot" geom2="floor" friction="0.5 0.5 0.01 0.001 0.001"/></contact>
</mujoco>"""


def test_explicit_pair_keeps_other_geoms_of_the_body():
    model = sim.Model.from_string(TWO_GEOM_BODY)
    cands = {tuple(sorted((int(a), int(b)))) for a, b in zip(model.pair_geom1, model.pair_geom2)}
    assert cands == {(0, 2)}, cands              # floor-knee dynamic; floor-foot only explicit
    b = sim.Batch(model, 4)
    b.step(100)
    q = b.get(sim.FIELD_QPOS)
    b.forward()
    g, _, _, _ = b.contacts(0)
    d = binding.OracleData(model)
    d.qpos[:] = q[0]
    d.forward()
    gr, _, _, _ = d.contacts()
    assert np.array_equal(g, gr), (g.tolist(), gr.tolist())
    pairs = {tuple(sorted(x)) for x in g.tolist()}
    assert (0, 2) in pairs and (0, 1) in pairs, pairs  # the knee on the floor (dynamic) and the foot (explicit)
    b.close()
