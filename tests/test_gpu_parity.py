"""GPU parity: the HIP path (libmrs.so through the C ABI) against the fp64 CPU oracle on the same
seeded inputs.  Tolerances (fp32 device arithmetic vs fp64 oracle; SURVEY.md §8d, BASELINE.json
north_star "qpos/qvel within 1e-5 rel"):

  qpos, qvel        |gpu - cpu| <= RTOL * max(|cpu|, SCALE)      RTOL = 1e-5 (1000-step rollouts)
  rangefinder       |gpu - cpu| <= 2e-5 * max(1, range) on >= 99.5% of rays (grazing hits at box
                    edges may switch faces) and identical hit/miss (-1) pattern
  depth image       |gpu - cpu| <= 1e-5 * depth on >= 99.9% of pixels (silhouette edges may flip)
  contacts          counts and the (geom1, geom2) list identical (integer work is bit-exact);
                    dist / pos / frame within 1e-4
"""
import numpy as np
import pytest

from conftest import ARM7, REF_SCENE
from flips import explain_flip
from mujoco_ros2_simulation_amd import sim, synth
import binding

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _oracle_rollout(model, qpos0, table, period, checkpoints, pre=None):
    """Per-env oracle rollout returning qpos/qvel/sensordata at each checkpoint (steps).  With `pre`
    (a dict), pre[c] receives each env's qpos at the start of step c - 1: mj_step evaluates the
    sensors in its forward() before integrating, so that is the pose the checkpoint's sensordata
    (rangefinder scans) was computed at."""
    n = qpos0.shape[0]
    out = {c: (np.zeros((n, model.nq)), np.zeros((n, model.nv)), np.zeros((n, model.nsensordata))) for c in checkpoints}
    if pre is not None:
        pre.update({c: np.zeros((n, model.nq)) for c in checkpoints})
    for e in range(n):
        d = binding.OracleData(model)
        d.qpos[:] = qpos0[e]
        t = 0
        for c in checkpoints:
            while t < c:
                if t % period == 0:
                    d.ctrl[:] = table[t // period, e]
                if pre is not None and t == c - 1:
                    pre[c][e] = d.qpos
                d.step()
                t += 1
            out[c][0][e] = d.qpos
            out[c][1][e] = d.qvel
            out[c][2][e] = d.sensordata
    return out


def _gpu_rollout(model, qpos0, table, period, checkpoints):
    n = qpos0.shape[0]
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, qpos0)
    out = {}
    t = 0
    for c in checkpoints:
        while t < c:
            b.set(sim.FIELD_CTRL, table[t // period])
            k = min(period - t % period, c - t)
            b.step(k)
            t += k
        out[c] = (b.get(sim.FIELD_QPOS), b.get(sim.FIELD_QVEL), b.get(sim.FIELD_SENSORDATA))
    b.close()
    return out


def _scale(x):
    return np.maximum(np.abs(x), 1.0)


def _quat_rot(q, v):
    w, x, y, z = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    return R @ v


def _grazing(model, qpos, sensor, delta=1e-4):
    """is rangefinder `sensor`'s ray within `delta` rad of a geom silhouette at `qpos`?  The oracle's
    mj_ray along the site's z axis is compared with rays tilted by +-delta about two axes normal to it:
    a ray that grazes an edge flips hit/miss or jumps to another surface (range changes by far more
    than the smooth delta * range * slope of a face it hits squarely)"""
    d = binding.OracleData(model)
    d.qpos[:] = qpos
    xpos, xquat, _, _ = d.kinematics()
    site = model.sensor_objid[sensor]
    b = model.site_bodyid[site]
    pnt = xpos[b] + _quat_rot(xquat[b], model.site_pos[site])
    sq = model.site_quat[site]
    w, x, y, z = sq
    bq = xquat[b]
    q = np.array([bq[0] * w - bq[1] * x - bq[2] * y - bq[3] * z, bq[0] * x + bq[1] * w + bq[2] * z - bq[3] * y,
                  bq[0] * y - bq[1] * z + bq[2] * w + bq[3] * x, bq[0] * z + bq[1] * y - bq[2] * x + bq[3] * w])
    vec = _quat_rot(q, np.array([0.0, 0.0, 1.0]))
    far = 50.0  # hits beyond this count as misses: a horizontal lidar ray tilted down by delta
    #             meets the infinite floor thousands of metres away, which is not a silhouette
    r0, _ = d.ray(pnt, vec, b)
    r0 = -1.0 if r0 > far else r0
    e1 = np.cross(vec, [1.0, 0, 0] if abs(vec[0]) < 0.9 else [0, 1.0, 0])
    e1 /= np.linalg.norm(e1)
    e2 = np.cross(vec, e1)
    for e in (e1, -e1, e2, -e2):
        v = vec + delta * e
        r, _ = d.ray(pnt, v / np.linalg.norm(v), b)
        r = -1.0 if r > far else r
        if (r < 0) != (r0 < 0):
            return True
        if r0 >= 0 and abs(r - r0) > 10 * delta * max(1.0, r0):
            return True
    return False


def _oracle_rollout_f32_state(model, qpos0, table, period, checkpoints):
    """the oracle's rollout with qpos/qvel rounded to fp32 after every step: how far fp32 storage of
    the state alone moves a trajectory from the fp64 one (the scene's own sensitivity)"""
    n = qpos0.shape[0]
    out = {c: np.zeros((n, model.nq)) for c in checkpoints}
    for e in range(n):
        d = binding.OracleData(model)
        d.qpos[:] = qpos0[e]
        t = 0
        for c in checkpoints:
            while t < c:
                if t % period == 0:
                    d.ctrl[:] = table[t // period, e]
                d.step()
                d.qpos[:] = d.qpos.astype(np.float32)
                d.qvel[:] = d.qvel.astype(np.float32)
                t += 1
            out[c][e] = d.qpos
    return out


GROUPS = [16, 32, 64]   # lanes per env; the batch picks one from nv and the env count, tests force each

# G = 16 workgroup layouts (batch.hip: waves per workgroup and helper waves are chosen per batch size).
# "auto" is what the batch picks for the test's env count (one-wave + helpers below one wave per SIMD);
# "wpb4" is the layout bench.py times on C3 (8192 envs: four-wave workgroups sharing the LDS ray
# tables, no helper waves -- step_kernel<16,false,false,false>); "wpb1" / "wpb1_help" are C4's layout
# without and with helper waves.  Other group widths have one layout.
LAYOUTS = {"auto": {}, "wpb4": {"MRS_G16_WPB": "4", "MRS_RAY_HELPERS": "0"},
           "wpb1": {"MRS_G16_WPB": "1", "MRS_RAY_HELPERS": "0"},
           "wpb1_help": {"MRS_G16_WPB": "1", "MRS_RAY_HELPERS": "1"}}
EXPECT = {"wpb4": (4, 0), "wpb1": (1, 0), "wpb1_help": (1, 1)}


def _layout_cases():
    out = []
    for g in GROUPS:
        for lay in (LAYOUTS if g == 16 else ["auto"]):
            out.append(pytest.param(g, lay, id=f"{g}-{lay}"))
    return out


def _apply_layout(monkeypatch, group, layout):
    monkeypatch.setenv("MRS_GROUP", str(group))
    for k in ("MRS_G16_WPB", "MRS_RAY_HELPERS"):
        monkeypatch.delenv(k, raising=False)
    for k, v in LAYOUTS[layout].items():
        monkeypatch.setenv(k, v)


def _check_layout(model, n, group, layout, has_rays):
    """the batch really runs the layout the case names (waves per workgroup, helper waves)"""
    if layout not in EXPECT:
        return
    b = sim.Batch(model, n)
    lay = b.layout()
    b.close()
    wpb, helpers = EXPECT[layout]
    assert lay["group"] == group and lay["waves_per_workgroup"] == wpb, lay
    assert lay["helper_waves"] == (helpers if has_rays else 0), lay


@pytest.mark.parametrize("group, layout", _layout_cases())
@pytest.mark.parametrize("scene, n_envs, steps", [(REF_SCENE, 64, 1000), (ARM7, 16, 1000)])
def test_rollout_parity(scene, n_envs, steps, group, layout, monkeypatch):
    _apply_layout(monkeypatch, group, layout)
    model = sim.Model.load(scene)
    envs = np.arange(n_envs)
    period = 10
    qpos0 = synth.initial_qpos(model, envs)
    table = synth.ctrl_table(model, envs, steps // period + 1, period)
    checkpoints = [1, 10, 100, steps]
    has_rays = any(model.sensor_type[i] == sim.SENS_RANGEFINDER for i in range(model.nsensor))
    _check_layout(model, n_envs, group, layout, has_rays)
    pre = {}
    ref = _oracle_rollout(model, qpos0, table, period, checkpoints, pre)
    got = _gpu_rollout(model, qpos0, table, period, checkpoints)
    _compare_rollout(model, scene.name, checkpoints, ref, got, pre)


def _compare_rollout(model, name, checkpoints, ref, got, pre):
    for c in checkpoints:
        q_ref, v_ref, s_ref = ref[c]
        q, v, s = got[c]
        eq = np.max(np.abs(q - q_ref) / _scale(q_ref))
        ev = np.max(np.abs(v - v_ref) / _scale(v_ref))
        print(f"{name} step {c}: max rel err qpos {eq:.2e} qvel {ev:.2e}")
        assert eq <= RTOL, f"qpos rel err {eq} at step {c}"
        assert ev <= RTOL, f"qvel rel err {ev} at step {c}"
        rf = np.array([i for i in range(model.nsensor) if model.sensor_type[i] == sim.SENS_RANGEFINDER])
        adr = model.sensor_adr[rf]
        # grazing rays (tangent to a sphere/capsule within rounding) may flip hit/miss
        flip = (s[:, adr] < 0) != (s_ref[:, adr] < 0)
        assert np.mean(flip) <= 0.002
        hit = (s_ref[:, adr] >= 0) & (s[:, adr] >= 0)
        err = np.zeros_like(s[:, adr])
        err[hit] = np.abs(s[:, adr][hit] - s_ref[:, adr][hit]) / np.maximum(1.0, s_ref[:, adr][hit])
        # a ray grazing a box edge may land on the adjacent face under a 1e-7 pose difference
        assert np.mean(err[hit] > 2e-5) <= 0.005, f"rangefinder mismatch fraction {np.mean(err[hit] > 2e-5)}"
        assert np.median(err[hit]) < 1e-6
        # every outlier and every hit/miss flip is a grazing ray: within 1e-4 rad of a silhouette
        bad = np.argwhere(flip | (err > 2e-5))
        for e, k in bad:  # (at the pose the scan was taken at: the start of the checkpoint's last step)
            assert _grazing(model, pre[c][e], rf[k]), (c, e, k, s[e, adr[k]], s_ref[e, adr[k]])
        print(f"  {len(bad)} rangefinder outliers / flips, all grazing a silhouette")


ARM7_1080 = ARM7.parent / "arm7_lidar1080.xml"


TWO_LIDARS = """<mujoco><compiler angle="radian"/><option timestep="0.002"/>
  <worldbody><geom type="plane" size="0 0 1"/>
    <geom type="box" pos="1.5 0 0.5" size="0.2 0.6 0.5"/>
    <geom type="sphere" pos="-1.2 0.8 0.6" size="0.3"/>
    <body name="lidar_a" pos="0 0 0.5" quat="0.5 0.5 0.5 0.5">
      <replicate count="90" sep="-" euler="0 0.0698132 0"><site name="ra"/></replicate>
    </body>
    <body name="lidar_b" pos="0.3 -0.4 0.7" quat="0.5 0.5 0.5 0.5">
      <replicate count="90" sep="-" euler="0 0.0698132 0"><site name="rb"/></replicate>
    </body>
    <body name="ball" pos="0.8 0.3 0.5"><freejoint/><geom type="sphere" size="0.15"/></body>
  </worldbody>
  <sensor><rangefinder name="la" site="ra"/><rangefinder name="lb" site="rb"/></sensor></mujoco>"""


def test_two_lidars_on_two_bodies():
    """two replicate-built lidars on different bodies: no single ray frame for the model (rays read
    from the model block), each pass still shares one lidar's body and origin; ranges against the
    oracle within 2e-5 on >= 99.5% of rays, hit / miss identical on >= 99.8%"""
    model = sim.Model.from_string(TWO_LIDARS)
    n = 8
    b = sim.Batch(model, n)
    assert b.layout()["rf_common"] == 0
    q = np.tile(model.qpos0, (n, 1))
    q[:, 0] += np.linspace(-0.3, 0.3, n)
    b.set(sim.FIELD_QPOS, q)
    b.forward()
    sd = b.get(sim.FIELD_SENSORDATA)
    b.close()
    same = close = total = 0
    for e in range(n):
        d = binding.OracleData(model)
        d.qpos[:] = q[e]
        d.forward()
        ref = d.sensordata
        same += int(np.sum((sd[e] >= 0) == (ref >= 0)))
        close += int(np.sum(np.abs(sd[e] - ref) <= 2e-5 * np.maximum(np.abs(ref), 1)))
        total += len(ref)
    assert same >= 0.998 * total and close >= 0.995 * total, (same, close, total)


def test_lidar1080_stays_on_16_lane_groups():
    """a 1080-beam lidar on C3's arm: the per-ray table no longer fits the two-workgroups-per-CU LDS
    budget, and the batch keeps its 16-lane groups (rays read from the model block) instead of
    falling to 32-lane groups; 300 steps within 1e-5 of the oracle, rangefinders as in
    test_rollout_parity"""
    model = sim.Model.load(ARM7_1080)
    b = sim.Batch(model, 16)
    lay = b.layout()
    b.close()
    print(lay)
    assert lay["group"] == 16
    n_envs, steps, period = 16, 300, 10
    envs = np.arange(n_envs)
    qpos0 = synth.initial_qpos(model, envs)
    table = synth.ctrl_table(model, envs, steps // period + 1, period)
    ref = _oracle_rollout(model, qpos0, table, period, [steps])
    got = _gpu_rollout(model, qpos0, table, period, [steps])
    q_ref, v_ref, s_ref = ref[steps]
    q, v, s = got[steps]
    assert np.max(np.abs(q - q_ref) / _scale(q_ref)) <= RTOL
    assert np.max(np.abs(v - v_ref) / _scale(v_ref)) <= RTOL
    rf = np.array([i for i in range(model.nsensor) if model.sensor_type[i] == sim.SENS_RANGEFINDER])
    adr = model.sensor_adr[rf]
    assert len(rf) == 1080
    flip = (s[:, adr] < 0) != (s_ref[:, adr] < 0)
    assert np.mean(flip) <= 0.002
    hit = (s_ref[:, adr] >= 0) & (s[:, adr] >= 0)
    err = np.abs(s[:, adr][hit] - s_ref[:, adr][hit]) / np.maximum(1.0, s_ref[:, adr][hit])
    assert np.mean(err > 2e-5) <= 0.005 and np.median(err) < 1e-6


@pytest.mark.parametrize("group", [16, 64])
def test_forward_lidar_closed_form(group, monkeypatch):
    monkeypatch.setenv("MRS_GROUP", str(group))
    """GPU rangefinders of the reference scene at qpos=0 equal 1.95/cos(0.3 - 0.025 i)."""
    model = sim.Model.load(REF_SCENE)
    b = sim.Batch(model, 8)
    b.forward()
    s = b.get(sim.FIELD_SENSORDATA)
    i = np.arange(24)
    np.testing.assert_allclose(s, np.tile(1.95 / np.cos(0.3 - 0.025 * i), (8, 1)), atol=2e-5)


def test_reference_position_pin_gpu():
    """robot_launch_test.py:112-132 on the GPU path: [0.5, -0.5] reached within 0.05 rad in 2 s."""
    model = sim.Model.load(REF_SCENE)
    b = sim.Batch(model, 4)
    b.set(sim.FIELD_CTRL, np.tile([0.5, -0.5], (4, 1)))
    for _ in range(100):  # 50 Hz controller writes, 10 physics steps each = 2 s
        b.step(10)
    q = b.get(sim.FIELD_QPOS)
    assert np.all(np.abs(q[:, 0] - 0.5) < 0.05) and np.all(np.abs(q[:, 1] + 0.5) < 0.05)
    np.testing.assert_allclose(b.get(sim.FIELD_TIME)[:, 0], 2.0, rtol=1e-12)


def test_full_size_batch_properties():
    """4096 envs (config C2 size): identical envs give identical results wherever they sit in the
    batch, results are deterministic across launches, and env 0 matches the oracle."""
    model = sim.Model.load(REF_SCENE)
    n = 4096
    qpos0 = np.tile(synth.initial_qpos(model, np.arange(4)), (n // 4, 1))
    ctrl = np.tile(synth.ctrl_table(model, np.arange(4), 1, 10)[0], (n // 4, 1))
    outs = []
    for _ in range(2):
        b = sim.Batch(model, n)
        b.set(sim.FIELD_QPOS, qpos0)
        b.set(sim.FIELD_CTRL, ctrl)
        b.step(200)
        outs.append(b.get(sim.FIELD_QPOS))
        b.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    q = outs[0].reshape(n // 4, 4, -1)
    assert np.all(q == q[:1])
    d = binding.OracleData(model)
    d.qpos[:] = qpos0[0]
    d.ctrl[:] = ctrl[0]
    d.step(200)
    np.testing.assert_allclose(outs[0][0], d.qpos, rtol=RTOL, atol=RTOL)


def test_depth_parity_reference_camera():
    model = sim.Model.load(REF_SCENE)
    b = sim.Batch(model, 2)
    q = np.array([[0.3, -0.7], [1.2, 0.4]])
    b.set(sim.FIELD_QPOS, q)
    b.forward()
    imgs = b.render_depth(0, 0, 2)
    for e in range(2):
        d = binding.OracleData(model)
        d.qpos[:] = q[e]
        d.forward()
        ref = d.render_depth(0)
        close = np.abs(imgs[e] - ref) <= 1e-5 * np.maximum(ref, 1)
        assert close.mean() >= 0.999, f"env {e}: {close.mean()}"


CONTACT_SCENE = """<mujoco><compiler angle="radian"/><option timestep="0.002" solver="PGS" iterations="50"/>
<worldbody><geom name="floor" type="plane" size="0 0 1" contype="3" conaffinity="3"/>
<geom name="ledge" type="box" pos="1 0 0.2" size="0.3 0.3 0.2"/>
<body pos="0 0 0.4"><freejoint/><geom type="sphere" size="0.1"/></body>
<body pos="1 0 0.8" euler="0.3 0.2 0"><freejoint/><geom type="capsule" size="0.05 0.2"/></body>
<body pos="-1 0 0.5" euler="0.1 0.2 0.3"><freejoint/><geom type="box" size="0.1 0.15 0.05" contype="2" conaffinity="2"/></body>
</worldbody></mujoco>"""


@pytest.mark.parametrize("group", [16, 64])
def test_contact_parity_short_horizon(group, monkeypatch):
    monkeypatch.setenv("MRS_GROUP", str(group))
    """Contact generation and PGS with free bodies: contact counts bit-exact, state within tolerance
    over a short horizon (contact dynamics diverge chaotically in fp32 vs fp64 over long ones)."""
    model = sim.Model.from_string(CONTACT_SCENE)
    b = sim.Batch(model, 4)
    d = binding.OracleData(model)
    for chunk in range(12):
        b.step(25)
        d.step(25)
        q = b.get(sim.FIELD_QPOS)[0]
        ncon = int(b.get(sim.FIELD_NCON)[0, 0])
        assert ncon == d.ncon, f"chunk {chunk}: ncon {ncon} vs {d.ncon}"
        np.testing.assert_allclose(q, d.qpos, atol=2e-3)
    assert d.ncon >= 3  # sphere on floor, capsule on ledge, box on floor (up to 4 corners)


def _contact_state(model, steps, n=4):
    """a state with contacts: seeded start, `steps` GPU steps under seeded actions (fp32 values)"""
    envs = np.arange(n)
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, synth.initial_qpos(model, envs))
    if model.nu:
        b.set(sim.FIELD_CTRL, synth.ctrl_table(model, envs, 1, 10)[0])
    if steps:
        b.step(steps)
    q = b.get(sim.FIELD_QPOS)
    b.close()
    return q


@pytest.mark.parametrize("scene, group, steps", [("contact", 16, 150), ("contact", 64, 150),
                                                 ("arm_boxes", 64, 30), ("arm_boxes", 64, 100)])
def test_contact_list_bit_exact(scene, group, steps, monkeypatch):
    """mjData.contact (mj_collision's output) after a forward pass from the same
    state on both sides: the (geom1, geom2) list equals the oracle's element by element (integer
    output: bit-exact, north_star), dist / pos / frame within 1e-4 (fp32 geometry).  States come from
    GPU steps, clear of contact thresholds: C5's start pose rests the boxes at exactly zero distance,
    where fp32 rounding of z decides whether a contact exists (SURVEY §7 'hard parts')"""
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = sim.Model.from_string(CONTACT_SCENE) if scene == "contact" else sim.Model.load(ARM_BOXES)
    qs = _contact_state(model, steps)
    b = sim.Batch(model, len(qs))
    b.set(sim.FIELD_QPOS, qs)
    b.forward()
    total = 0
    for e, q in enumerate(qs):
        g, dist, pos, frame = b.contacts(e)
        d = binding.OracleData(model)
        d.qpos[:] = q
        d.forward()
        g_ref, dist_ref, pos_ref, frame_ref = d.contacts()
        assert g.shape == g_ref.shape and np.array_equal(g, g_ref), (e, g.tolist(), g_ref.tolist())
        np.testing.assert_allclose(dist, dist_ref, atol=1e-4)
        np.testing.assert_allclose(pos, pos_ref, atol=1e-4)
        np.testing.assert_allclose(frame, frame_ref, atol=1e-4)
        total += len(g)
    b.close()
    assert total >= 3 * len(qs)


def test_full_size_c3_batch_properties():
    """8192 envs of the C3 arm + 360-ray lidar (BASELINE configs[2] size): envs with equal inputs
    give bit-identical state and scans wherever they sit in the batch, launches are deterministic,
    and env 0 matches the oracle after 100 steps"""
    model = sim.Model.load(ARM7)
    n, reps = 8192, 8
    q0 = np.tile(synth.initial_qpos(model, np.arange(reps)), (n // reps, 1))
    ctrl = np.tile(synth.ctrl_table(model, np.arange(reps), 1, 10)[0], (n // reps, 1))
    outs = []
    for _ in range(2):
        b = sim.Batch(model, n)
        b.set(sim.FIELD_QPOS, q0)
        b.set(sim.FIELD_CTRL, ctrl)
        b.step(100)
        outs.append((b.get(sim.FIELD_QPOS), b.get(sim.FIELD_SENSORDATA)))
        b.close()
    for a, c in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, c)
    q, s = outs[0]
    assert np.all(q.reshape(n // reps, reps, -1) == q[:reps][None])
    assert np.all(s.reshape(n // reps, reps, -1) == s[:reps][None])
    d = binding.OracleData(model)
    d.qpos[:] = q0[0]
    d.ctrl[:] = ctrl[0]
    d.step(100)
    np.testing.assert_allclose(q[0], d.qpos, rtol=RTOL, atol=RTOL)


def test_full_size_c3_1000_steps_vs_oracle(monkeypatch):
    """the exact kernel bench.py times on C3 (8192 envs: G = 16, four-wave workgroups with the shared
    LDS ray tables, no helper waves) held to the 1000-step pin: 64 distinct envs (synthetic initial
    states and Philox ctrl tables), tiled over the batch, against the oracle within 1e-5; every copy
    of an env identical to the first wherever it sits"""
    for k in ("MRS_GROUP", "MRS_G16_WPB", "MRS_RAY_HELPERS"):
        monkeypatch.delenv(k, raising=False)
    model = sim.Model.load(ARM7)
    n, reps, steps, period = 8192, 64, 1000, 10
    envs = np.arange(reps)
    q0 = synth.initial_qpos(model, envs)
    table = synth.ctrl_table(model, envs, steps // period + 1, period)
    b = sim.Batch(model, n)
    lay = b.layout()
    assert lay["group"] == 16 and lay["waves_per_workgroup"] == 4 and lay["helper_waves"] == 0, lay
    b.set(sim.FIELD_QPOS, np.tile(q0, (n // reps, 1)))
    checkpoints = [1, 10, 100, steps]
    got, t = {}, 0
    for c in checkpoints:
        while t < c:
            b.set(sim.FIELD_CTRL, np.tile(table[t // period], (n // reps, 1)))
            k = min(period - t % period, c - t)
            b.step(k)
            t += k
        q, v, s = b.get(sim.FIELD_QPOS), b.get(sim.FIELD_QVEL), b.get(sim.FIELD_SENSORDATA)
        for x in (q, v, s):
            assert np.all(x.reshape(n // reps, reps, -1) == x[:reps][None]), c
        got[c] = (q[:reps], v[:reps], s[:reps])
    b.close()
    pre = {}
    ref = _oracle_rollout(model, q0, table, period, checkpoints, pre)
    _compare_rollout(model, "c3-8192", checkpoints, ref, got, pre)


def test_abi_errors_leave_batch_usable():
    """error behaviour of the C ABI on a live batch (int status codes, message via
    mrs_last_error, no exceptions across the ABI): out-of-range env ranges, n_steps < 1, a bad
    camera index and an out-of-range contact env all fail with MRS_ERR_INVALID, and the batch
    still steps afterwards"""
    model = sim.Model.load(REF_SCENE)
    b = sim.Batch(model, 3)
    bad = [lambda: b.get(sim.FIELD_QPOS, 2, 2), lambda: b.set(sim.FIELD_QPOS, np.zeros((4, 2))),
           lambda: b.step(0), lambda: b.contacts(3), lambda: b.reset(-1, 1, 5),
           lambda: b.get_device(sim.FIELD_TIME, 1)]
    for call in bad:
        with pytest.raises(sim.MrsError) as ei:
            call()
        assert ei.value.code == -1 and str(ei.value)
    img = np.zeros((480, 640), dtype=np.float32)
    assert sim.lib().mrs_batch_render_depth(b._h, 5, 0, 1, img.ctypes.data) == -1  # no camera 5
    assert b"camera" in sim.lib().mrs_last_error()
    b.step(5)
    assert np.all(np.isfinite(b.get(sim.FIELD_QPOS)))
    assert b.contacts(0)[0].shape == (0, 2)  # the reference scene has no contact pairs
    b.close()


@pytest.mark.parametrize("group", [16, 64])
def test_autoreset_on_nan(group, monkeypatch):
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = sim.Model.load(REF_SCENE)
    b = sim.Batch(model, 3)
    q = np.zeros((3, 2))
    q[1, 0] = np.nan
    b.set(sim.FIELD_QPOS, q)
    b.step(1)
    w = b.get(sim.FIELD_WARNING)
    assert w[1, 0] == 1 and w[0, 0] == 0 and w[2, 0] == 0
    assert np.all(np.isfinite(b.get(sim.FIELD_QPOS)))


IMU_FT = ARM7.parent / "imu_ft.xml"


@pytest.mark.parametrize("group", [16, 64])
def test_imu_ft_sensor_parity(group, monkeypatch):
    """row f2: framequat/gyro/accelerometer/force/torque (mj_rnePostConstraint + mj_sensorAcc) on the
    GPU against the oracle over a seeded rollout with motor torques and a box landing on the floor
    (contact forces enter cfrc_ext).  Acceleration-level outputs tolerate 1e-3 of their scale: they
    difference nearly balanced fp32 forces."""
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = sim.Model.load(IMU_FT)
    n, steps, period = 16, 400, 10
    envs = np.arange(n)
    qpos0 = synth.initial_qpos(model, envs)
    table = synth.ctrl_table(model, envs, steps // period + 1, period)
    checkpoints = [1, 50, 200, steps]
    ref = _oracle_rollout(model, qpos0, table, period, checkpoints)
    got = _gpu_rollout(model, qpos0, table, period, checkpoints)
    for c in checkpoints:
        q_ref, v_ref, s_ref = ref[c]
        q, v, s = got[c]
        assert np.max(np.abs(q - q_ref) / _scale(q_ref)) <= 1e-4, c
        for i in range(model.nsensor):
            a, dim = model.sensor_adr[i], model.sensor_dim[i]
            sr, sg = s_ref[:, a:a + dim], s[:, a:a + dim]
            scale = max(1.0, float(np.max(np.abs(sr))))
            err = float(np.max(np.abs(sg - sr))) / scale
            assert err <= 1e-3, (c, model.id2name(sim.OBJ_SENSOR, i), err)


MOBILE = ARM7.parent / "mobile_base.xml"


@pytest.mark.parametrize("group", [16, 64])
def test_mobile_base_parity(group, monkeypatch):
    """config C4: free-joint base driven by two sphere wheels (velocity actuators, pyramidal friction
    contacts), 32-beam lidar and a 640x480 depth frame, GPU vs oracle over a seeded rollout.
    The caster's stick-slip contact (50 unconverged PGS sweeps) is chaotic: rounding the oracle's own
    state to fp32 after each step moves it ~1e-4 from the fp64 trajectory by step 100.  So: 1e-5 over
    the first 10 steps; later, the GPU must be no further from the fp64 oracle than 10x that fp32
    rounding sensitivity (+1e-5).  The 1e-5 per-step pin is test_gpu_solvers::test_reseeded_step_parity."""
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = sim.Model.load(MOBILE)
    n, steps, period = 8, 500, 10
    envs = np.arange(n)
    qpos0 = synth.initial_qpos(model, envs)
    table = synth.ctrl_table(model, envs, steps // period + 1, period)
    checkpoints = [10, 100, steps]
    ref = _oracle_rollout(model, qpos0, table, period, checkpoints)
    chaos = _oracle_rollout_f32_state(model, qpos0, table, period, checkpoints)
    got = _gpu_rollout(model, qpos0, table, period, checkpoints)
    for c in checkpoints:
        q_ref, v_ref, s_ref = ref[c]
        q, v, s = got[c]
        err = np.max(np.abs(q - q_ref) / _scale(q_ref))
        sens = np.max(np.abs(chaos[c] - q_ref) / _scale(q_ref))
        print(f"mobile step {c}: qpos rel err {err:.2e} (fp32-state sensitivity {sens:.2e})")
        assert err <= (1e-5 if c <= 10 else 10 * sens + 1e-5), (c, err, sens)
    # moving: the base left its start
    assert np.all(np.linalg.norm(ref[steps][0][:, :2] - qpos0[:, :2], axis=1) > 1e-3)
    # depth of env 0 at the end of the rollout against the oracle's render of the GPU state
    b = sim.Batch(model, 1)
    b.set(sim.FIELD_QPOS, got[steps][0][:1])
    b.forward()
    depth = b.render_depth(0, 0, 1)[0]
    d = binding.OracleData(model)
    d.qpos[:] = got[steps][0][0]
    d.forward()
    want = d.render_depth(0)
    close = np.isclose(depth, want, rtol=1e-5, atol=1e-5)
    assert depth.shape == (480, 640) and close.mean() >= 0.999
    b.close()


ARM_BOXES = ARM7.parent / "arm_boxes.xml"


@pytest.mark.parametrize("group", [64])
def test_contact_rich_parity(group, monkeypatch):
    """config C5: 7-DoF arm, floor and 8 free boxes (two stacked pairs): nv = 55, 32 contacts
    (plane-box and box-box, pyramidal friction), ~135 PGS rows at the 50-iteration cap.  Contact
    counts must match exactly.  The unconverged PGS amplifies rounding, so the rollout bound is the
    scene's own fp32 sensitivity (the oracle with its state rounded to fp32 every step): the GPU
    within 10x of it + 1e-5; 1e-5 after one step.  The 1e-5 per-step pin over 200 steps is
    test_gpu_solvers::test_reseeded_step_parity."""
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = sim.Model.load(ARM_BOXES)
    n, steps, period = 4, 200, 10
    envs = np.arange(n)
    qpos0 = synth.initial_qpos(model, envs)
    table = synth.ctrl_table(model, envs, steps // period + 1, period)
    checkpoints = [1, 20, steps]
    ref = _oracle_rollout(model, qpos0, table, period, checkpoints)
    chaos = _oracle_rollout_f32_state(model, qpos0, table, period, checkpoints)
    got = _gpu_rollout(model, qpos0, table, period, checkpoints)
    for c in checkpoints:
        err = np.max(np.abs(got[c][0] - ref[c][0]) / _scale(ref[c][0]))
        sens = np.max(np.abs(chaos[c] - ref[c][0]) / _scale(ref[c][0]))
        print(f"arm_boxes step {c}: qpos rel err {err:.2e} (fp32-state sensitivity {sens:.2e})")
        assert err <= (1e-5 if c == 1 else 10 * sens + 1e-5), (c, err, sens)
    # contact counts (integer work, bit-exact): 24 at the start (the stacked boxes start 2 mm
    # apart), 40 at step 200 (box-box face contacts give every vertex of the clipped polygon)
    for q, want in ((qpos0[0], 24), (ref[steps][0][0], 40)):
        b = sim.Batch(model, 1)
        b.set(sim.FIELD_QPOS, q[None])
        b.forward()
        d = binding.OracleData(model)
        d.qpos[:] = q
        d.forward()
        assert int(b.get(sim.FIELD_NCON)[0, 0]) == d.ncon == want
        b.close()


def test_box_stack_rests(monkeypatch):
    """box-box: a rotated box resting on a box resting on the floor stays stacked on the GPU"""
    xml = """<mujoco><option timestep="0.002"/><worldbody><geom type="plane" size="0 0 1"/>
    <body pos="0 0 0.1"><freejoint/><geom type="box" size="0.1 0.1 0.1" mass="1"/></body>
    <body pos="0.03 0.02 0.32" euler="0 0 0.4"><freejoint/><geom type="box" size="0.1 0.1 0.1" mass="1"/></body>
    </worldbody></mujoco>"""
    model = sim.Model.from_string(xml)
    b = sim.Batch(model, 4)
    b.step(1000)
    q = b.get(sim.FIELD_QPOS)
    np.testing.assert_allclose(q[:, 2], 0.1, atol=5e-4)
    np.testing.assert_allclose(q[:, 9], 0.3, atol=1e-3)
    assert np.all(b.get(sim.FIELD_NCON)[:, 0] == 8)
    d = binding.OracleData(model)
    d.step(1000)
    np.testing.assert_allclose(q[0], d.qpos, atol=1e-4)
    b.close()


def test_tall_stack_fallback_solver(monkeypatch):
    """blocked mode with one island larger than the register-resident solve (a tower of five boxes:
    4 box-box faces of 8 contacts (the clipped octagons of boxes turned 0.2 rad) + 4 plane-box
    contacts, 4 rows each = 144 rows in one island, > 48 rows per pipe):
    the global-record path must give the oracle's trajectory and contact counts"""
    monkeypatch.setenv("MRS_GROUP", "64")
    bodies = "".join(
        f'<body pos="0 0 {0.1 + 0.2 * k + 0.001 * k:.4f}" euler="0 0 {0.2 * k:.2f}"><freejoint/>'
        f'<geom type="box" size="0.1 0.1 0.1" mass="1"/></body>' for k in range(5))
    xml = f"""<mujoco><option timestep="0.002" solver="PGS"/><worldbody><geom type="plane" size="0 0 1"/>{bodies}
    </worldbody></mujoco>"""
    model = sim.Model.from_string(xml)
    b = sim.Batch(model, 2)
    lay = b.layout()
    assert lay["blocked"] == 1 and lay["group"] == 64
    d = binding.OracleData(model)
    # while the tower settles the trajectories agree to fp32 rounding; afterwards the unconverged
    # 100-iteration PGS of the 80-row island amplifies rounding (measured: the register-resident path
    # built with room for 80 rows drifts from the oracle just as much), so only the rest pose and the
    # contact counts are pinned at 200 steps
    b.step(40)
    d.step(40)
    np.testing.assert_allclose(b.get(sim.FIELD_QPOS)[0], d.qpos, atol=5e-5)
    b.step(160)
    q = b.get(sim.FIELD_QPOS)
    ncon = b.get(sim.FIELD_NCON)[:, 0]
    b.close()
    d.step(160)
    assert int(ncon[0]) == d.ncon == 36
    np.testing.assert_allclose(q[0], d.qpos, atol=5e-3)
    # soft contacts: each layer sinks ~1 mm under the boxes above it (pyramid R = 2 mu^2 R / impratio)
    np.testing.assert_allclose(q[0, 2::7], [0.1 + 0.2 * k for k in range(5)], atol=6e-3)


@pytest.mark.parametrize("condim, levels", [(1, "rows"), (3, "items")])
def test_blocked_register_paths(condim, levels, monkeypatch):
    """the two register-resident blocked solves on one-island towers of aligned boxes (4 contacts per
    face): three boxes with condim 3 give 12 four-row contact items (the item-blocked solve's limit);
    four boxes with condim 1 give 16 one-row items, more than 12 but within the row-level solve's 48
    rows.  50 steps against the oracle"""
    monkeypatch.setenv("MRS_GROUP", "64")
    bodies = "".join(
        f'<body pos="0 0 {0.1 + 0.2 * k + 0.001 * k:.4f}"><freejoint/>'
        f'<geom type="box" size="0.1 0.1 0.1" mass="1" condim="{condim}"/></body>' for k in range(3 if condim == 3 else 4))
    xml = f"""<mujoco><option timestep="0.002" solver="PGS" iterations="50"/><worldbody>
    <geom type="plane" size="0 0 1" condim="{condim}"/>{bodies}</worldbody></mujoco>"""
    model = sim.Model.from_string(xml)
    b = sim.Batch(model, 2)
    assert b.layout()["blocked"] == 1
    d = binding.OracleData(model)
    b.step(50)
    d.step(50)
    q = b.get(sim.FIELD_QPOS)
    ncon = b.get(sim.FIELD_NCON)[:, 0]
    b.close()
    assert int(ncon[0]) == d.ncon
    assert d.ncon == (12 if condim == 3 else 16)
    np.testing.assert_allclose(q[0], d.qpos, atol=5e-5)
    np.testing.assert_allclose(q[1], d.qpos, atol=5e-5)


@pytest.mark.parametrize("v1", [False, True])
def test_depth_all_primitives(v1, monkeypatch):
    """depth render of every primitive type (plane, sphere, capsule, cylinder, ellipsoid, rotated box,
    one box enclosing nothing but partly off-screen, one geom behind the camera) against the oracle's
    render, with the per-frame (v2) and the per-tile (v1) kernel"""
    if v1:
        monkeypatch.setenv("MRS_DEPTH_V1", "1")
    xml = """<mujoco><worldbody>
      <geom type="plane" size="0 0 1"/>
      <geom type="sphere" size="0.3" pos="0.6 -0.4 0.3"/>
      <geom type="capsule" size="0.1 0.3" pos="-0.5 0.2 0.4" euler="23 11 0"/>
      <geom type="cylinder" size="0.2 0.25" pos="0.1 0.6 0.25"/>
      <geom type="ellipsoid" size="0.3 0.15 0.2" pos="-0.1 -0.6 0.2" euler="0 0 40"/>
      <geom type="box" size="0.2 0.1 0.3" pos="0.5 0.5 0.3" euler="17 29 52"/>
      <geom type="box" size="0.3 0.3 0.3" pos="-1.4 -0.2 0.3"/>
      <geom type="sphere" size="0.2" pos="0 -3.5 1.5"/>
      <camera name="cam" pos="0 -2 1.2" euler="63 0 0" fovy="60" resolution="320 240"/>
    </worldbody></mujoco>"""
    model = sim.Model.from_string(xml)
    b = sim.Batch(model, 2)
    b.forward()
    img = b.render_depth(0, 0, 2)
    b.close()
    d = binding.OracleData(model)
    d.forward()
    want = d.render_depth(0)
    for e in range(2):
        close = np.isclose(img[e], want, rtol=1e-5, atol=1e-5)
        assert img[e].shape == (240, 320) and close.mean() >= 0.999, close.mean()
    # every primitive is visible somewhere in the frame
    assert len(np.unique(np.round(want, 2))) > 50


def test_rgbd_all_primitives():
    """colour pass (mrs_batch_render_rgbd) on coloured primitives against the oracle's
    orc_render_rgbd: depth identical to render_depth, each channel within 1 (u8 rounding) except at
    silhouettes and box edges where fp32 picks the other geom or face (<= 1% of pixels)"""
    xml = """<mujoco><worldbody>
      <geom type="plane" size="0 0 1" rgba="0.6 0.6 0.6 1"/>
      <geom type="sphere" size="0.3" pos="0.6 -0.4 0.3" rgba="1 0 0 1"/>
      <geom type="capsule" size="0.1 0.3" pos="-0.5 0.2 0.4" euler="23 11 0" rgba="0 1 0 1"/>
      <geom type="cylinder" size="0.2 0.25" pos="0.1 0.6 0.25" rgba="0 0 1 1"/>
      <geom type="ellipsoid" size="0.3 0.15 0.2" pos="-0.1 -0.6 0.2" euler="0 0 40" rgba="1 1 0 1"/>
      <geom type="box" size="0.2 0.1 0.3" pos="0.5 0.5 0.3" euler="17 29 52" rgba="0 1 1 1"/>
      <camera name="cam" pos="0 -2 1.2" euler="63 0 0" fovy="60" resolution="320 240"/>
    </worldbody></mujoco>"""
    model = sim.Model.from_string(xml)
    b = sim.Batch(model, 2)
    b.forward()
    depth, rgb = b.render_rgbd(0, 0, 2)
    np.testing.assert_array_equal(depth, b.render_depth(0, 0, 2))
    b.close()
    d = binding.OracleData(model)
    d.forward()
    wd, wrgb = d.render_rgbd(0)
    for e in range(2):
        diff = np.abs(rgb[e].astype(int) - wrgb.astype(int)).max(axis=-1)
        assert (diff <= 1).mean() >= 0.99, (diff <= 1).mean()
    assert len({tuple(c) for c in wrgb.reshape(-1, 3)[::97]}) > 20  # shaded, not flat


def test_camera_pipeline_snapshot():
    """mrs_batch_render_async renders the poses of the step it was queued after (its snapshot), while
    the following steps move the bodies: frames equal a synchronous render of that same state, and
    colour equals the synchronous colour pass"""
    import torch
    from conftest import ROOT
    model = sim.Model.load(ROOT / "scenes" / "mobile_base.xml")
    n = 64
    envs = np.arange(n)
    W, H = (int(v) for v in model.cam_resolution[0])
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, synth.initial_qpos(model, envs))
    b.set(sim.FIELD_CTRL, synth.ctrl_table(model, envs, 1, 10)[0])
    b.step(30)
    want = torch.empty((n, H, W), dtype=torch.float32, device="cuda")
    want_rgb = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda")
    b.render_rgbd_device(0, 0, n, want.data_ptr(), want_rgb.data_ptr())
    b.sync()
    got = torch.full((n, H, W), -7.0, dtype=torch.float32, device="cuda")
    got_rgb = torch.zeros((n, H, W, 3), dtype=torch.uint8, device="cuda")
    b.render_async(0, 0, n, got.data_ptr(), got_rgb.data_ptr())
    b.step(50)                       # moves the base while the frame renders
    b.render_wait()
    b.sync()
    assert torch.equal(got, want)
    assert torch.equal(got_rgb, want_rgb)
    # a second frame after more steps differs (the snapshot is refreshed), and again matches
    b.render_async(0, 0, n, got.data_ptr(), 0)
    b.sync()
    b.render_depth_device(0, 0, n, want.data_ptr())
    b.sync()
    assert torch.equal(got, want)
    b.close()


def _reseeded_sensors(model, n, steps, period=10, settle=0):
    """every GPU step starts from the oracle's fp64 state rounded to fp32 (qpos, qvel,
    qacc_warmstart, ctrl), given identically to a second oracle instance; returns per sensor the
    worst |gpu - oracle| over all env-steps and the sensor's largest |oracle value|, plus the worst
    relative qpos / qvel errors and the contact-count mismatches"""
    envs = np.arange(n)
    qpos0 = synth.initial_qpos(model, envs)
    table = synth.ctrl_table(model, envs, (steps + settle) // period + 1, period)
    orc = [binding.OracleData(model) for _ in envs]
    ref = [binding.OracleData(model) for _ in envs]
    for e, d in enumerate(orc):
        d.qpos[:] = qpos0[e]
    for t in range(settle):
        for e, d in enumerate(orc):
            if t % period == 0 and model.nu:
                d.ctrl[:] = table[t // period, e]
            d.step()
    b = sim.Batch(model, n)
    err = np.zeros(model.nsensor)
    mag = np.zeros(model.nsensor)
    wq = wv = 0.0
    flips, unexplained = 0, []
    for t in range(settle, settle + steps):
        for e, (d, r) in enumerate(zip(orc, ref)):
            if t % period == 0 and model.nu:
                d.ctrl[:] = table[t // period, e]
            for k in ("qpos", "qvel", "qacc_warmstart", "ctrl"):
                getattr(r, k)[:] = getattr(d, k).astype(np.float32)
        for f, k in ((sim.FIELD_QPOS, "qpos"), (sim.FIELD_QVEL, "qvel"), (sim.FIELD_QACC_WARMSTART, "qacc_warmstart"),
                     (sim.FIELD_CTRL, "ctrl")):
            b.set(f, np.array([getattr(r, k) for r in ref]))
        start = [(r.qpos.copy(), r.qvel.copy()) for r in ref]
        b.step(1)
        for d, r in zip(orc, ref):
            r.step()
            d.step()
        nc, nr = b.get(sim.FIELD_NCON)[:, 0].astype(int), np.array([r.ncon for r in ref])
        ok = nc == nr
        flips += int(np.sum(~ok))
        for e in np.flatnonzero(~ok):  # each excluded env-step must be a threshold case (tests/flips.py)
            done, diff, _ = explain_flip(model, *start[e], b.contacts(int(e))[0])
            if not done:
                unexplained.append((t, int(e), diff))
        s, sr = b.get(sim.FIELD_SENSORDATA)[ok], np.array([r.sensordata for r in ref])[ok]
        q, v = b.get(sim.FIELD_QPOS)[ok], b.get(sim.FIELD_QVEL)[ok]
        qr, vr = np.array([r.qpos for r in ref])[ok], np.array([r.qvel for r in ref])[ok]
        if ok.any():
            wq = max(wq, float(np.max(np.abs(q - qr) / _scale(qr))))
            wv = max(wv, float(np.max(np.abs(v - vr) / _scale(vr))))
            for i in range(model.nsensor):
                a, dim = model.sensor_adr[i], model.sensor_dim[i]
                err[i] = max(err[i], float(np.max(np.abs(s[:, a:a + dim] - sr[:, a:a + dim]))))
                mag[i] = max(mag[i], float(np.max(np.abs(sr[:, a:a + dim]))))
    b.close()
    assert not unexplained, unexplained[:5]
    return err, mag, wq, wv, flips


@pytest.mark.parametrize("group", [16, 64])
def test_imu_ft_reseeded_1e5(group, monkeypatch):
    """row f2 at the north-star tolerance: framequat / gyro / accelerometer / force / torque (what
    read() maps, reference src/mujoco_system_interface.cpp:1069-1095) after every one of 200
    re-seeded steps (motor torques, a box landing on the floor) within 1e-5 of each sensor's scale --
    the same bound as qpos / qvel.  Re-seeding removes the trajectory divergence that the 400-step
    rollout test (test_imu_ft_sensor_parity) has to tolerate.
    Scale: max(1, largest |value|), except force sensors, whose scale is the force they balance:
    max(1, largest |value|, subtree mass x |g|).  A force sensor on a free body (box_force) reads the
    body's net unbalanced force, 0 in exact arithmetic; what either side reports is the solver's
    residual, which in fp32 is eps x cond(H) x the forces in balance (the body's weight against its
    contact forces), ~1e-6 of them after the Newton refinement step -- not a fraction of a zero."""
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = sim.Model.load(IMU_FT)
    err, mag, wq, wv, flips = _reseeded_sensors(model, 16, 200)
    scale = np.maximum(mag, 1.0)
    for i in range(model.nsensor):
        if model.sensor_type[i] == sim.SENS_FORCE:
            body = model.site_bodyid[model.sensor_objid[i]]
            scale[i] = max(scale[i], float(model.body_subtreemass[body]) * 9.81)
    rel = err / scale
    for i in range(model.nsensor):
        print(f"{model.id2name(sim.OBJ_SENSOR, i):14s} max |err| {err[i]:.2e}  scale {scale[i]:.3g}  rel {rel[i]:.2e}")
    print(f"qpos {wq:.2e} qvel {wv:.2e} flips {flips}")
    assert flips <= 0.01 * 16 * 200
    assert wq <= 1e-5 and wv <= 1e-5
    worst = int(np.argmax(rel))
    assert rel.max() <= 1e-5, (model.id2name(sim.OBJ_SENSOR, worst), rel.max())


@pytest.mark.parametrize("group", [16, 64])
def test_contact_parity_reseeded_1e5(group, monkeypatch):
    """CONTACT_SCENE (sphere, capsule on a ledge, box; PGS 50) over 300 re-seeded steps: contact
    counts equal (at most 1% of env-steps excepted, a contact at fp32 rounding distance of its
    threshold) and qpos / qvel within 1e-5 of scale per step -- test_contact_parity_short_horizon's
    2e-3 is the free-running divergence, not the per-step arithmetic"""
    monkeypatch.setenv("MRS_GROUP", str(group))
    model = sim.Model.from_string(CONTACT_SCENE)
    err, mag, wq, wv, flips = _reseeded_sensors(model, 8, 300)
    print(f"G={group}: qpos {wq:.2e} qvel {wv:.2e} flips {flips}")
    assert flips <= 0.01 * 8 * 300
    assert wq <= 1e-5 and wv <= 1e-5


def _tiled_inputs(model, n, reps):
    q0 = np.tile(synth.initial_qpos(model, np.arange(reps)), (n // reps, 1))
    ctrl = np.tile(synth.ctrl_table(model, np.arange(reps), 1, 10)[0], (n // reps, 1))
    return q0, ctrl


def _oracle_pair(model, q0, ctrl, steps):
    """env 0 on the oracle in fp64 and with its state rounded to fp32 after every step (the scene's
    own sensitivity to fp32 storage: the contact-rich configs are chaotic over tens of steps)"""
    out = []
    for rnd in (False, True):
        d = binding.OracleData(model)
        d.qpos[:] = q0
        d.ctrl[:] = ctrl
        for _ in range(steps):
            d.step()
            if rnd:
                d.qpos[:] = d.qpos.astype(np.float32)
                d.qvel[:] = d.qvel.astype(np.float32)
        out.append(d)
    return out


def test_full_size_c4_batch_properties():
    """2048 envs of C4 (mobile base + 32-beam lidar + 640x480 depth camera: BASELINE configs[3] per
    GPU) with a depth frame of every env: envs with equal inputs give bit-identical state, scans and
    frames wherever they sit in the batch, launches are deterministic, env 0's state stays within the
    scene's fp32 sensitivity of the oracle (10x + 1e-5, as test_mobile_base_parity) and its frame
    equals the oracle's render of the same state (1e-5 on >= 99.9% of pixels)."""
    import torch
    model = sim.Model.load(MOBILE)
    n, reps, steps = 2048, 8, 100
    q0, ctrl = _tiled_inputs(model, n, reps)
    W, H = model.cam_resolution[0]
    outs = []
    for _ in range(2):
        b = sim.Batch(model, n)
        b.set(sim.FIELD_QPOS, q0)
        b.set(sim.FIELD_CTRL, ctrl)
        for _ in range(steps // 10):
            b.step(10)
        # (after mj_step the poses are those of the step's start; forward() brings them to the final
        # qpos, the state the oracle renders below)
        b.forward()
        frames = torch.empty((n, H, W), dtype=torch.float32, device="cuda")
        b.render_depth_device(0, 0, n, frames.data_ptr())
        b.sync()
        outs.append((b.get(sim.FIELD_QPOS), b.get(sim.FIELD_SENSORDATA), frames))
        b.close()
    (q, s, f), (q2, s2, f2) = outs
    np.testing.assert_array_equal(q, q2)
    np.testing.assert_array_equal(s, s2)
    assert torch.equal(f, f2)
    assert np.all(q.reshape(n // reps, reps, -1) == q[:reps][None])
    assert np.all(s.reshape(n // reps, reps, -1) == s[:reps][None])
    fr = f.view(n // reps, reps, H, W)
    assert bool((fr == fr[:1]).all())
    ref, ref32 = _oracle_pair(model, q0[0], ctrl[0], steps)
    scale = np.maximum(np.abs(ref.qpos), 1.0)
    err, sens = np.max(np.abs(q[0] - ref.qpos) / scale), np.max(np.abs(ref32.qpos - ref.qpos) / scale)
    print(f"C4 env 0 after {steps} steps: qpos err {err:.2e}, fp32-state sensitivity {sens:.2e}")
    assert err <= 10 * sens + 1e-5
    d = binding.OracleData(model)
    d.qpos[:] = q[0]
    d.forward()
    img = d.render_depth(0)
    close = np.abs(f[0].cpu().numpy() - img) <= 1e-5 * np.maximum(img, 1)
    assert close.mean() >= 0.999, close.mean()


def test_c2_bench_variant():
    """the exact workload `bench.py --config c2` times: the reference scene with <flag
    sensor="disable"/> (bench.ref_scene_xml), its default solver (Newton), 4096 envs, ctrl from the
    bench's Philox table changed every 10-step period.  Identical envs identical wherever they sit,
    deterministic across launches, sensordata never written (sensors disabled), and the four distinct
    envs against the oracle after 1000 steps within 1e-5 (qpos / qvel, relative to max(|x|, 1))."""
    import bench
    xml, base = bench.ref_scene_xml(sensors=False)
    model = sim.Model.from_string(xml, base)
    assert model.solver == 2 and model.disableflags & (1 << 12)  # Newton; mjDSBL_SENSOR
    n, period, steps, k = 4096, 10, 1000, 4
    ids = np.arange(k)
    q0 = synth.initial_qpos(model, ids)
    tab = synth.ctrl_table(model, ids, steps // period, period)
    outs = []
    for _ in range(2):
        b = sim.Batch(model, n)
        b.set(sim.FIELD_QPOS, np.tile(q0, (n // k, 1)))
        for p in range(steps // period):
            b.set(sim.FIELD_CTRL, np.tile(tab[p], (n // k, 1)))
            b.step(period)
        outs.append((b.get(sim.FIELD_QPOS), b.get(sim.FIELD_QVEL), b.get(sim.FIELD_SENSORDATA)))
        b.close()
    for a, c in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, c)
    q, v, sd = outs[0]
    assert np.all(q.reshape(n // k, k, -1) == q[None, :k]) and np.all(v.reshape(n // k, k, -1) == v[None, :k])
    assert np.all(sd == 0)
    for e in range(k):
        d = binding.OracleData(model)
        d.qpos[:] = q0[e]
        for p in range(steps // period):
            d.ctrl[:] = tab[p, e]
            d.step(period)
        for got, ref in ((q[e], d.qpos), (v[e], d.qvel)):
            err = np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1.0))
            assert err <= RTOL, (e, err)


