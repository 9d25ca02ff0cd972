"""Pins the fp64 CPU oracle (oracle/oracle.c) before it is trusted as the parity checker:
closed-form known answers and the reference's behavioural pin
(test/src/robot_launch_test.py:112-132).  MuJoCo itself is not available anywhere in this pipeline
(SURVEY.md §8c), so beyond these pins the oracle is 'parity unpinned' against upstream mj_step."""
from pathlib import Path

import numpy as np
import pytest

from mujoco_ros2_simulation_amd import sim
import binding


def test_lidar_ranges_closed_form(s2_model):
    d = binding.OracleData(s2_model)
    d.forward()
    i = np.arange(24)
    expect = 1.95 / np.cos(0.3 - 0.025 * i)  # every ray hits the upper arm's y=+0.05 face
    # the MJCF quaternions are rounded to ~1e-6, which shifts ranges by < 1e-5
    np.testing.assert_allclose(d.sensordata, expect, atol=1e-5)
    # values printed in SURVEY.md Appendix B
    np.testing.assert_allclose(d.sensordata[[0, 11, 12, 23]], [2.041168, 1.950610, 1.950000, 2.026129], atol=2e-6)


@pytest.mark.parametrize("q2", [0.0, 0.4, -1.3, 2.5])
def test_mass_matrix_closed_form(s2_model, q2):
    d = binding.OracleData(s2_model)
    d.qpos[:] = [0.7, q2]
    M = d.mass_matrix()
    c = np.cos(q2)
    expect = np.array([[0.45 + 27 * (1.25 + c) + 6.75, 0.225 + 27 * (0.25 + 0.5 * c)],
                       [0.225 + 27 * (0.25 + 0.5 * c), 6.975]])
    np.testing.assert_allclose(M, expect, rtol=1e-12)


SERVO = """<mujoco><compiler angle="radian"/><option timestep="0.002" integrator="{integ}" gravity="0 0 -9.81"/>
<worldbody><body><joint name="j" axis="0 0 1" damping="{b}"/>
<inertial pos="0 0 0" mass="1" diaginertia="{I} {I} {I}"/></body></worldbody>
<actuator><position joint="j" kp="{kp}" kv="{kv}"/></actuator></mujoco>"""


@pytest.mark.parametrize("integ", ["Euler", "implicitfast"])
def test_servo_recurrence(integ):
    I, b, kp, kv, h, c = 0.5, 0.3, 40.0, 2.0, 0.002, 0.8
    m = sim.Model.from_string(SERVO.format(integ=integ, b=b, I=I, kp=kp, kv=kv))
    d = binding.OracleData(m)
    d.ctrl[:] = [c]
    q, v = 0.0, 0.0
    for _ in range(300):
        f = kp * (c - q) - (b + kv) * v
        a = f / (I + h * (b if integ == "Euler" else b + kv))
        v = v + h * a
        q = q + h * v
        d.step()
        assert d.qpos[0] == pytest.approx(q, rel=1e-12, abs=1e-14)
        assert d.qvel[0] == pytest.approx(v, rel=1e-12, abs=1e-14)
    assert d.time == pytest.approx(300 * h)


def test_ballistic_free_body():
    xml = """<mujoco><option timestep="0.01"/><worldbody><body pos="0 0 5"><freejoint/>
    <geom type="sphere" size="0.1" contype="0" conaffinity="0"/></body></worldbody></mujoco>"""
    m = sim.Model.from_string(xml)
    d = binding.OracleData(m)
    d.qvel[:] = [1.0, -0.5, 2.0, 0, 0, 3.0]  # translation + spin about z
    h, g, n = 0.01, 9.81, 100
    d.step(n)
    # semi-implicit Euler: v_n = v0 - n h g, z_n = z0 + h sum_k v_k
    z = 5 + h * sum(2.0 - k * h * g for k in range(1, n + 1))
    assert d.qpos[2] == pytest.approx(z, rel=1e-12)
    assert d.qpos[0] == pytest.approx(1.0 * n * h) and d.qpos[1] == pytest.approx(-0.5 * n * h)
    # spin about the body z axis: quaternion (cos(wt/2), 0, 0, sin(wt/2))
    ang = 3.0 * n * h
    np.testing.assert_allclose(d.qpos[3:], [np.cos(ang / 2), 0, 0, np.sin(ang / 2)], atol=1e-12)


def test_reference_position_pin(s2_model):
    """robot_launch_test.py:112-132: command [0.5, -0.5]; after 2 s |q - cmd| < 0.05."""
    d = binding.OracleData(s2_model)
    d.ctrl[:] = [0.5, -0.5]
    d.step(1000)  # 2 s at the default 0.002 s timestep
    assert abs(d.qpos[0] - 0.5) < 0.05 and abs(d.qpos[1] + 0.5) < 0.05
    assert d.nefc >= 1  # joint1 friction loss row is always present


PLANE_CAM = """<mujoco><compiler angle="radian"/><statistic extent="1"/><visual><map znear="0.01" zfar="50"/></visual><worldbody>
<geom type="plane" size="0 0 1" {tilt}/>
<camera name="c" pos="0 0 {z0}" fovy="60" resolution="64 48"/></worldbody></mujoco>"""


def test_depth_plane_constant():
    z0 = 1.7
    m = sim.Model.from_string(PLANE_CAM.format(z0=z0, tilt=""))
    d = binding.OracleData(m)
    d.forward()
    img = d.render_depth(0)
    np.testing.assert_allclose(img, z0, rtol=1e-6)  # eye-space z, not Euclidean range


def _slopes(H, W, fovy=60):
    f = 0.5 * H / np.tan(np.radians(fovy / 2))
    x = (np.arange(W) + 0.5 - 0.5 * W) / f
    y = (0.5 * H - np.arange(H) - 0.5) / f
    return x[None, :] + 0 * y[:, None], y[:, None] + 0 * x[None, :]


def _u8(c):
    return np.floor(np.clip(c, 0, 1) * 255 + 0.5).astype(np.uint8)


def test_rgb_plane_point_light():
    """colour KAT (lit model, oracle.c lit_color): a plane (rgba 0.8 0.5 0.2, material specular 0.5
    shininess 0.25) seen straight down from height z0, lit only by a point light at the camera
    (headlight off, no attenuation, 90-degree cone, exponent 0).  Pixel slope (x, y): the light
    direction has N.L = cos = 1/sqrt(1 + x^2 + y^2); the half vector with the view axis gives
    N.H = sqrt((1 + cos) / 2), so colour = base (0.1 + 0.6 cos) + 0.3 * 0.5 (N.H)^32; the depth is
    unchanged by the colour pass"""
    z0 = 1.7
    xml = PLANE_CAM.format(z0=z0, tilt='material="m" rgba="0.8 0.5 0.2 1"').replace(
        "<worldbody>", '<asset><material name="m" specular="0.5" shininess="0.25"/></asset><worldbody>'
        f'<light pos="0 0 {z0}" dir="0 0 -1" directional="false" cutoff="90" exponent="0" attenuation="1 0 0" '
        'ambient="0.1 0.1 0.1" diffuse="0.6 0.6 0.6" specular="0.3 0.3 0.3" castshadow="false"/>').replace(
        "<visual>", '<visual><headlight active="0"/>')
    m = sim.Model.from_string(xml)
    d = binding.OracleData(m)
    d.forward()
    depth, rgb = d.render_rgbd(0)
    np.testing.assert_array_equal(depth, d.render_depth(0))
    x, y = _slopes(*depth.shape)
    cos = 1 / np.sqrt(1 + x ** 2 + y ** 2)
    spec = 0.15 * np.sqrt((1 + cos) / 2) ** 32
    want = np.array([0.8, 0.5, 0.2]) * (0.1 + 0.6 * cos)[..., None] + spec[..., None]
    assert np.abs(rgb.astype(int) - _u8(want).astype(int)).max() <= 1
    assert (rgb == _u8(want)).mean() > 0.99


def test_rgb_sphere_centre_and_sky():
    """a sphere in front of the camera under the default headlight (ambient 0.1, diffuse 0.4,
    specular 0.5; default material specular 0.5): the centre pixel faces the ray, N.L = N.H = 1, so
    colour = 0.5 rgba + 0.25; rays that miss are black without a skybox, and show the gradient skybox
    rgb2 + (rgb1 - rgb2) (1 + d_z) / 2 of the world ray direction with one"""
    xml = """<mujoco>{asset}<worldbody>
      <geom type="sphere" size="0.2" pos="0 0 -1" rgba="0.2 0.4 1 1"/>
      <camera name="c" pos="0 0 0" fovy="60" resolution="65 49"/></worldbody></mujoco>"""
    d = binding.OracleData(sim.Model.from_string(xml.format(asset="")))
    d.forward()
    depth, rgb = d.render_rgbd(0)
    np.testing.assert_array_equal(rgb[24, 32], _u8(0.5 * np.array([0.2, 0.4, 1]) + 0.25))
    assert depth[24, 32] == pytest.approx(0.8, rel=1e-6)
    np.testing.assert_array_equal(rgb[0, 0], [0, 0, 0])
    sky = '<asset><texture type="skybox" builtin="gradient" rgb1="0.4 0.6 0.8" rgb2="0 0.2 0" width="8" height="8"/></asset>'
    d = binding.OracleData(sim.Model.from_string(xml.format(asset=sky)))
    d.forward()
    depth, rgb = d.render_rgbd(0)
    x, y = _slopes(*depth.shape)
    dz = -1 / np.sqrt(1 + x ** 2 + y ** 2)
    c1, c2 = np.array([0.4, 0.6, 0.8]), np.array([0, 0.2, 0])
    want = _u8(c2 + (c1 - c2) * (0.5 * (1 + dz))[..., None])
    miss = depth >= depth.max()
    assert miss.mean() > 0.9
    assert np.abs(rgb[miss].astype(int) - want[miss].astype(int)).max() <= 1


def test_rgb_directional_shadow():
    """shadow KAT: plane z = 0 seen from (0, 0, 3), a sphere (r 0.2, centre (0, 0, 0.5)) and a
    directional castshadow light along (1, 0, -1)/sqrt(2) (headlight off): a plane point P is in shadow
    iff its ray towards the light, -(1, 0, -1)/sqrt(2), passes within 0.2 of the centre; there the
    colour is the ambient base * 0.2, elsewhere base * (0.2 + 0.5 / sqrt(2)) (N.L = 1/sqrt(2), no
    specular).  Pixels within 2 mm of the shadow edge and pixels that see the sphere are skipped."""
    xml = """<mujoco><visual><headlight active="0"/></visual><worldbody>
      <light directional="true" dir="1 0 -1" castshadow="true" ambient="0.2 0.2 0.2" diffuse="0.5 0.5 0.5" specular="0 0 0"/>
      <geom type="plane" size="0 0 1" rgba="1 0.5 0.25 1"/>
      <geom type="sphere" size="0.2" pos="0 0 0.5" rgba="0 1 0 1"/>
      <camera name="c" pos="0 0 3" fovy="60" resolution="96 72"/></worldbody></mujoco>"""
    d = binding.OracleData(sim.Model.from_string(xml))
    d.forward()
    depth, rgb = d.render_rgbd(0)
    x, y = _slopes(*depth.shape)
    on_plane = np.abs(depth - 3) < 1e-6
    P = np.stack([3 * x, 3 * y, np.zeros_like(x)], -1)
    L = np.array([-1, 0, 1]) / np.sqrt(2)
    v = np.array([0, 0, 0.5]) - P
    s = v @ L
    dist = np.sqrt(np.maximum((v ** 2).sum(-1) - s ** 2, 0))
    shadow = (dist < 0.2) & (s > 0)
    clear = on_plane & (np.abs(dist - 0.2) > 2e-3)
    base = np.array([1, 0.5, 0.25])
    want = np.where(shadow[..., None], base * 0.2, base * (0.2 + 0.5 / np.sqrt(2)))
    assert shadow[clear].sum() > 50 and (~shadow[clear]).sum() > 1000
    assert np.abs(rgb[clear].astype(int) - _u8(want)[clear].astype(int)).max() <= 1


def test_rgb_checker_texture():
    """builtin checker texture on a plane (texuniform, texrepeat 1 1, 2 x 2 blocks of rgb1 / rgb2 per
    unit length): plane point (u, v) shows rgb1 when frac(u) < 0.5 and frac(v) < 0.5 or both >= 0.5,
    else rgb2; material specular 0 under the default headlight: colour = 0.5 * texel"""
    xml = """<mujoco><asset>
      <texture name="t" type="2d" builtin="checker" rgb1="0.9 0.9 0.9" rgb2="0.2 0.3 0.4" width="64" height="64"/>
      <material name="m" texture="t" texrepeat="1 1" texuniform="true" specular="0"/></asset><worldbody>
      <geom type="plane" size="0 0 1" material="m"/>
      <camera name="c" pos="0.1 0.2 2" fovy="60" resolution="80 60"/></worldbody></mujoco>"""
    d = binding.OracleData(sim.Model.from_string(xml))
    d.forward()
    depth, rgb = d.render_rgbd(0)
    x, y = _slopes(*depth.shape)
    u, v = 0.1 + 2 * x, 0.2 + 2 * y
    fu, fv = u - np.floor(u), v - np.floor(v)
    first = (fu < 0.5) == (fv < 0.5)
    clear = (np.abs(fu - 0.5) > 0.02) & (np.abs(fv - 0.5) > 0.02) & (fu > 0.02) & (fu < 0.98) & (fv > 0.02) & (fv < 0.98)
    want = _u8(0.5 * np.where(first[..., None], [0.9, 0.9, 0.9], [0.2, 0.3, 0.4]))
    assert first[clear].sum() > 100 and (~first[clear]).sum() > 100
    np.testing.assert_array_equal(rgb[clear], want[clear])


def test_depth_tilted_plane_rows():
    z0, alpha = 2.0, 0.2
    m = sim.Model.from_string(PLANE_CAM.format(z0=z0, tilt=f'euler="{alpha} 0 0"'))
    d = binding.OracleData(m)
    d.forward()
    img = d.render_depth(0)
    H, W = img.shape
    f = 0.5 * H / np.tan(np.radians(30))
    rows = np.arange(H)
    y = (0.5 * H - rows - 0.5) / f  # camera-frame y of each row at z = -1
    # plane through the origin with normal (0, -sin a, cos a); ray (x, y, -1) t from (0, 0, z0)
    t = z0 * np.cos(alpha) / (np.cos(alpha) + y * np.sin(alpha))
    np.testing.assert_allclose(img[:, W // 2], t, rtol=1e-6)
    assert np.allclose(img, img[:, :1])  # depth constant along rows


@pytest.mark.parametrize("geom, hit", [
    ('type="sphere" size="0.5"', 2.5), ('type="box" size="0.3 0.4 0.5"', 2.7),
    ('type="capsule" size="0.2 0.5" euler="0 1.5707963267948966 0"', 2.3),
    ('type="cylinder" size="0.25 0.5" euler="0 1.5707963267948966 0"', 2.5),
    ('type="capsule" size="0.2 0.5"', 2.8), ('type="cylinder" size="0.25 0.5"', 2.75),
    ('type="ellipsoid" size="0.1 0.6 0.3"', 2.9),
])
def test_ray_primitives(geom, hit):
    xml = f'<mujoco><compiler angle="radian"/><worldbody><geom {geom}/></worldbody></mujoco>'
    m = sim.Model.from_string(xml)
    d = binding.OracleData(m)
    d.forward()
    dist, gid = d.ray([-3.0, 0, 0], [1.0, 0, 0])
    assert gid == 0 and dist == pytest.approx(hit, abs=1e-6)
    dist, gid = d.ray([-3.0, 5, 0], [1.0, 0, 0])
    assert gid == -1 and dist == -1


def test_contact_sphere_on_plane():
    xml = """<mujoco><option timestep="0.002"/><worldbody><geom type="plane" size="0 0 1"/>
    <body pos="0 0 0.5"><freejoint/><geom type="sphere" size="0.1"/></body></worldbody></mujoco>"""
    m = sim.Model.from_string(xml)
    d = binding.OracleData(m)
    d.step(1500)
    # the sphere comes to rest on the plane with a small soft-contact penetration
    assert d.qpos[2] == pytest.approx(0.1, abs=3e-3)
    assert abs(d.qvel[2]) < 1e-2
    assert d.ncon == 1
    g, dist, pos, frame = d.contacts()
    assert list(g[0]) == [0, 1]
    np.testing.assert_allclose(frame[0, :3], [0, 0, 1], atol=1e-12)


# ---------------------------------------------------------------- IMU / force-torque (row f2)
IMU_FT = Path(__file__).resolve().parents[1] / "scenes" / "imu_ft.xml"


def _sens(m, d, name):
    from mujoco_ros2_simulation_amd import sim
    i = m.name2id(sim.OBJ_SENSOR, name)
    a = m.sensor_adr[i]
    return d.sensordata[a:a + m.sensor_dim[i]].copy()


def _quat2mat(q):
    w, x, y, z = q
    return np.array([[w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z]])


def test_acc_sensors_welded_body_at_rest():
    """a body welded to the world: accelerometer = R' (0,0,g); force = m R' (0,0,g) (the support);
    torque about the site = R' ((c - p) x f)  (mj_sensorAcc conventions)"""
    from mujoco_ros2_simulation_amd import sim
    m = sim.Model.load(IMU_FT)
    d = binding.OracleData(m)
    d.forward()
    Rb = _quat2mat([0.9238795, 0, 0.3826834, 0])
    Rs = _quat2mat([0.7071068, 0.7071068, 0, 0])
    R = Rb @ Rs
    g = np.array([0, 0, 9.81])
    f = 2.0 * g
    c = np.array([0.5, 0.5, 1.0])
    p = c + Rb @ np.array([0.1, 0, 0.05])
    np.testing.assert_allclose(_sens(m, d, "fixed_accel"), R.T @ g, atol=1e-5)
    np.testing.assert_allclose(_sens(m, d, "fixed_force"), R.T @ f, atol=1e-5)
    np.testing.assert_allclose(_sens(m, d, "fixed_torque"), R.T @ np.cross(c - p, f), atol=1e-5)


def test_acc_sensors_free_fall_and_rest_on_floor():
    """free fall reads zero specific force; resting on the floor the accelerometer reads +g and the
    free body's interaction force is ~0 (gravity balanced by the contact: cfrc_ext sign)"""
    from mujoco_ros2_simulation_amd import sim
    m = sim.Model.load(IMU_FT)
    d = binding.OracleData(m)
    d.forward()
    np.testing.assert_allclose(_sens(m, d, "box_accel"), 0, atol=1e-9)
    np.testing.assert_allclose(_sens(m, d, "box_force"), 0, atol=1e-9)
    d.step(2000)
    np.testing.assert_allclose(_sens(m, d, "box_accel"), [0, 0, 9.81], atol=2e-3)
    assert np.linalg.norm(_sens(m, d, "box_force")) < 1e-3 * 1.5 * 9.81


# ---------------------------------------------------------------- friction (pyramidal, condim 3)
_SLIDE = """<mujoco><option timestep="0.002"/><worldbody><geom type="plane" size="0 0 1"/>
<body pos="0 0 0.1"><freejoint/><geom type="{g}" size="{s}" mass="1"/></body></worldbody></mujoco>"""


def test_friction_box_stops_at_mu_g():
    """a box launched at 1 m/s on mu = 1 stops after ~v0^2 / (2 mu g) = 5.1 cm along either tangent
    direction (both pyramid edges use the sliding coefficient; the impulsive start makes the
    pyramidal contact hop, so the bounds are loose)"""
    for axis in (0, 1):
        m = sim.Model.from_string(_SLIDE.format(g="box", s="0.1 0.1 0.1"))
        d = binding.OracleData(m)
        d.step(200)
        x0 = d.qpos[axis]
        d.qvel[axis] = 1.0
        d.step(150)  # 0.3 s
        assert abs(d.qvel[axis]) < 0.01
        assert 0.03 < d.qpos[axis] - x0 < 0.1


def test_friction_sphere_rolls_at_five_sevenths():
    """a solid sphere launched sliding settles into rolling without slip at v = 5/7 v0"""
    m = sim.Model.from_string(_SLIDE.format(g="sphere", s="0.1"))
    d = binding.OracleData(m)
    d.step(200)
    d.qvel[0] = 1.0
    d.step(500)
    assert abs(d.qvel[0] - 5 / 7) < 0.01
    assert abs(d.qvel[4] * 0.1 - d.qvel[0]) < 0.01   # rolling: omega r = v


def _rk4_step(f, x, h):
    k1 = f(x)
    k2 = f(x + 0.5 * h * k1)
    k3 = f(x + 0.5 * h * k2)
    k4 = f(x + h * k3)
    return x + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)


def test_servo_rk4_closed_form():
    """mj_RungeKutta(4) on a damped position servo: every force is explicit under RK4 (joint damping
    and the actuator's kv included), so each step is the classic RK4 map of q' = v,
    v' = (kp (c - q) - (b + kv) v) / I"""
    I, b, kp, kv, h, c = 0.5, 0.3, 40.0, 2.0, 0.002, 0.8
    m = sim.Model.from_string(SERVO.format(integ="RK4", b=b, I=I, kp=kp, kv=kv))
    d = binding.OracleData(m)
    d.ctrl[:] = [c]
    f = lambda x: np.array([x[1], (kp * (c - x[0]) - (b + kv) * x[1]) / I])  # noqa: E731
    x = np.zeros(2)
    for _ in range(300):
        x = _rk4_step(f, x, h)
        d.step()
        assert d.qpos[0] == pytest.approx(x[0], rel=1e-12, abs=1e-14)
        assert d.qvel[0] == pytest.approx(x[1], rel=1e-12, abs=1e-14)
    assert d.time == pytest.approx(300 * h)


def test_ballistic_free_body_rk4():
    """RK4 integrates constant gravity exactly (z = z0 + v t - g t^2 / 2) and a constant spin of an
    isotropic body exactly (no gyroscopic torque)"""
    xml = """<mujoco><option timestep="0.01" integrator="RK4"/><worldbody><body pos="0 0 5"><freejoint/>
    <geom type="sphere" size="0.1" contype="0" conaffinity="0"/></body></worldbody></mujoco>"""
    m = sim.Model.from_string(xml)
    d = binding.OracleData(m)
    d.qvel[:] = [1.0, -0.5, 2.0, 0, 0, 3.0]
    h, g, n = 0.01, 9.81, 100
    d.step(n)
    t = n * h
    assert d.qpos[2] == pytest.approx(5 + 2.0 * t - 0.5 * g * t * t, rel=1e-12)
    assert d.qvel[2] == pytest.approx(2.0 - g * t, rel=1e-12)
    assert d.qpos[0] == pytest.approx(1.0 * t) and d.qpos[1] == pytest.approx(-0.5 * t)
    ang = 3.0 * t
    np.testing.assert_allclose(d.qpos[3:], [np.cos(ang / 2), 0, 0, np.sin(ang / 2)], atol=1e-12)


@pytest.mark.parametrize("q2, v", [(0.4, (1.3, -0.7)), (-1.1, (0.2, 2.5)), (2.0, (-3.0, 0.5))])
def test_bias_velocity_derivative_closed_form(s2_model, q2, v):
    """the full implicit integrator's RNE derivative (orc_bias_vel, mjd_rne_vel restated) on the
    reference's 2-link arm: its hinges are parallel to gravity, so qfrc_bias is the planar Coriolis /
    centrifugal force of link 2 (mass m2 = 27, com lc2 = 0.5 from the elbow, link 1 l1 = 1):
    bias = h (-(2 v1 v2 + v2^2), v1^2), h = m2 l1 lc2 sin q2 -- independent of the link inertias -- so
    d bias / d v = h [[-2 v2, -2 (v1 + v2)], [2 v1, 0]]"""
    d = binding.OracleData(s2_model)
    d.qpos[:] = [0.3, q2]
    d.qvel[:] = v
    d.forward()
    hh = 27 * 1.0 * 0.5 * np.sin(q2)
    v1, v2 = v
    expect = hh * np.array([[-2 * v2, -2 * (v1 + v2)], [2 * v1, 0.0]])
    np.testing.assert_allclose(d.bias_vel(), expect, atol=1e-9)


def test_servo_recurrence_implicit():
    """a single hinge about its own principal axis has no velocity-dependent bias force, so the full
    implicit integrator reduces to implicitfast's recurrence (a = f / (I + h (b + kv)))"""
    I, b, kp, kv, h, c = 0.5, 0.3, 40.0, 2.0, 0.002, 0.8
    m = sim.Model.from_string(SERVO.format(integ="implicit", b=b, I=I, kp=kp, kv=kv))
    d = binding.OracleData(m)
    d.ctrl[:] = [c]
    q, v = 0.0, 0.0
    for _ in range(300):
        f = kp * (c - q) - (b + kv) * v
        v = v + h * f / (I + h * (b + kv))
        q = q + h * v
        d.step()
        assert d.qpos[0] == pytest.approx(q, rel=1e-12, abs=1e-14)
        assert d.qvel[0] == pytest.approx(v, rel=1e-12, abs=1e-14)


def test_implicit_two_link_step(s2_model):
    """one implicit step of the free-swinging 2-link arm (no actuation) in closed form: the velocity
    update solves (M + h (diag(damping) + d bias / d v)) a = qfrc_smooth + qfrc_constraint with the
    closed-form mass matrix and Coriolis derivative, the joints' damping and the position servos' kv
    (no joint limit is active; the friction-loss row of joint 1 enters through the oracle's own
    qfrc_constraint)"""
    xml = (Path(__file__).resolve().parent / "golden" / "ref_scenes" / "scene.xml").read_text()
    xml = xml.replace('<include file="test_robot.xml"/>', '<include file="test_robot.xml"/><option integrator="implicit"/>')
    m = sim.Model.from_string(xml, str(Path(__file__).resolve().parent / "golden" / "ref_scenes"))
    assert m.integrator == 2
    d = binding.OracleData(m)
    q, v = np.array([0.2, 0.9]), np.array([1.5, -2.0])
    d.qpos[:] = q
    d.qvel[:] = v
    d.forward()
    qacc = d.qacc.copy()
    a_s, f_s = d.smooth()
    M = d.mass_matrix()
    hh = 27 * 0.5 * np.sin(q[1])
    dB = hh * np.array([[-2 * v[1], -2 * (v[0] + v[1])], [2 * v[0], 0.0]])
    damp = np.array([m.dof_damping[0], m.dof_damping[1]], dtype=float)
    bias = np.asarray(m.actuator_biasprm).reshape(m.nu, -1)
    for a in range(m.nu):  # position servos: d(actuator force)/d(qvel) = biasprm[2] = -kv
        damp[m.jnt_dofadr[m.actuator_trnid[a][0]]] -= bias[a, 2]
    h = m.timestep
    qfrc_con = M @ (qacc - a_s)   # the constraint force from mj_fwdConstraint's qacc
    a_int = np.linalg.solve(M + h * (np.diag(damp) + dB), f_s + qfrc_con)
    d.step()
    np.testing.assert_allclose(d.qvel, v + h * a_int, rtol=1e-10, atol=1e-12)


def test_equality_kats():
    """equality constraints in the oracle against closed forms: a free body hung by a connect at its
    origin swings exactly like the same body on a ball joint (when the ball is supported) or keeps its
    anchor within the soft constraint's sag; a body welded to another keeps the relative pose while
    the pair tumbles; a joint coupling q1 = 2 q2 holds within the soft constraint's error"""
    from mujoco_ros2_simulation_amd import sim
    import binding
    xml_c = """<mujoco><option timestep="0.001"/><worldbody>
    <body name="b" pos="0 0 1"><freejoint/><geom type="box" size="0.05 0.05 0.2" pos="0.1 0 -0.2" mass="1"/></body></worldbody>
    <equality><connect body1="b" anchor="0 0 0" solref="0.005 1"/></equality></mujoco>"""
    d = binding.OracleData(sim.Model.from_string(xml_c))
    for _ in range(1000):
        d.step()
    assert np.max(np.abs(d.qpos[:3] - [0, 0, 1])) < 1e-4          # the anchor stays put (soft: ~2.5e-5 sag)
    assert abs(d.qpos[5]) > 0.02                                    # and the box swings about it
    xml2 = """<mujoco><option timestep="0.001"/><worldbody>
    <body name="a" pos="0 0 1"><freejoint/><geom type="box" size="0.1 0.1 0.1" mass="1"/></body>
    <body name="b" pos="0.25 0 1" euler="0 0 30"><freejoint/><geom type="sphere" size="0.05" mass="0.5"/></body></worldbody>
    <equality><weld body1="a" body2="b"/></equality></mujoco>"""
    d = binding.OracleData(sim.Model.from_string(xml2))
    d.qvel[:] = [0, 0, 0, 1, 2, 3, 0, 0, 0, 0, 0, 0]
    for _ in range(300):
        d.step()
    qa, qb = d.qpos[:7], d.qpos[7:]
    w, x, y, z = qa[3:]
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    np.testing.assert_allclose(R.T @ (qb[:3] - qa[:3]), [0.25, 0, 0], atol=5e-4)
    c = np.array([w, -x, -y, -z])
    rel = np.array([c[0] * qb[3] - c[1] * qb[4] - c[2] * qb[5] - c[3] * qb[6], c[0] * qb[4] + c[1] * qb[3] + c[2] * qb[6] - c[3] * qb[5],
                    c[0] * qb[5] - c[1] * qb[6] + c[2] * qb[3] + c[3] * qb[4], c[0] * qb[6] + c[1] * qb[5] - c[2] * qb[4] + c[3] * qb[3]])
    np.testing.assert_allclose(rel * np.sign(rel[0]), [np.cos(np.pi / 12), 0, 0, np.sin(np.pi / 12)], atol=1e-3)
    xml_j = """<mujoco><option timestep="0.002"/><worldbody>
    <body name="a"><joint name="j1" axis="0 0 1"/><geom type="capsule" size="0.02 0.1" fromto="0 0 0 0.2 0 0"/></body>
    <body name="b" pos="0 0.5 0"><joint name="j2" axis="0 0 1"/><geom type="capsule" size="0.02 0.1" fromto="0 0 0 0.2 0 0"/></body></worldbody>
    <equality><joint joint1="j1" joint2="j2" polycoef="0 2 0 0 0" solref="0.005 1"/></equality>
    <actuator><position joint="j2" kp="10"/></actuator></mujoco>"""
    d = binding.OracleData(sim.Model.from_string(xml_j))
    d.ctrl[:] = 0.3
    worst, reach = 0.0, 0.0
    for _ in range(2000):
        d.step()
        worst = max(worst, abs(d.qpos[0] - 2 * d.qpos[1]))
        reach = max(reach, d.qpos[1])
    assert worst < 5e-3 and reach > 0.2  # the driven joint swings to the target; the coupled one follows


# ---------------------------------------------------------------- polytope face contacts (multiccd)
_CUBE = 'vertex="-1 -1 -1 1 -1 -1 1 1 -1 -1 1 -1 -1 -1 1 1 -1 1 1 1 1 -1 1 1" scale="0.1 0.1 0.1"'


def _face_scene(extra_bodies: str) -> str:
    return f"""<mujoco><compiler angle="radian"/><asset><mesh name="cube" {_CUBE}/></asset>
    <worldbody><geom name="table" type="box" pos="0 0 -0.05" size="1 1 0.05"/>{extra_bodies}</worldbody></mujoco>"""


def test_mesh_cube_resting_flat_gets_four_corner_contacts(built):
    """a mesh cube (half size 0.1) resting flat on a box, sunk by 1 mm: the face contacts are its four
    bottom corners, each at distance -1e-3 from the table top, positioned midway (z = -5e-4), normal
    +z from the table (geom1, the lower type) to the cube; without the face contacts
    (RESTATE_NO_MULTICCD) MPR gives one contact"""
    import binding
    from mujoco_ros2_simulation_amd import sim
    m = sim.Model.from_string(_face_scene('<body pos="0.3 -0.2 0.099"><freejoint/><geom type="mesh" mesh="cube"/></body>'))
    d = binding.OracleData(m)
    d.forward()
    g, dist, pos, fr = d.contacts()
    assert len(g) == 4 and all(tuple(x) == (0, 1) for x in g.tolist())
    np.testing.assert_allclose(dist, -1e-3, atol=1e-12)
    np.testing.assert_allclose(fr[:, :3], np.tile([0, 0, 1.0], (4, 1)), atol=1e-12)
    want = {(0.3 + sx * 0.1, -0.2 + sy * 0.1) for sx in (-1, 1) for sy in (-1, 1)}
    got = {(round(p[0], 9), round(p[1], 9)) for p in pos}
    assert got == {(round(x, 9), round(y, 9)) for x, y in want}
    np.testing.assert_allclose(pos[:, 2], -5e-4, atol=1e-12)
    m.set_restate(sim.RESTATE_NO_MULTICCD)
    d = binding.OracleData(m)
    d.forward()
    assert len(d.contacts()[0]) == 1


def test_mesh_cube_tipped_on_edge_and_stacked(built):
    """a cube tipped by 0.1 rad about x resting on its lower edge gets the edge's two ends (the other
    two bottom corners are ~2 cm above the table, beyond margin); a cube stacked flat on another cube
    (mesh-mesh, 1 mm overlap, shifted by 2 cm in x) gets the four corners of the overlap rectangle"""
    import binding
    from mujoco_ros2_simulation_amd import sim
    th = 0.1
    z = 0.1 * np.cos(th) + 0.1 * np.sin(th) - 1e-3  # lowest edge 1 mm into the table
    m = sim.Model.from_string(_face_scene(
        f'<body pos="0 0 {z:.12f}" euler="{th} 0 0"><freejoint/><geom type="mesh" mesh="cube"/></body>'))
    d = binding.OracleData(m)
    d.forward()
    g, dist, pos, fr = d.contacts()
    assert len(g) == 2, (g, dist)
    np.testing.assert_allclose(dist, -1e-3, atol=1e-9)
    np.testing.assert_allclose(sorted(pos[:, 0]), [-0.1, 0.1], atol=1e-9)
    m = sim.Model.from_string(_face_scene(
        '<body pos="0 0 0.1"><freejoint/><geom type="mesh" mesh="cube"/></body>'
        '<body pos="0.02 0 0.299"><freejoint/><geom type="mesh" mesh="cube"/></body>'))
    d = binding.OracleData(m)
    d.forward()
    g, dist, pos, fr = d.contacts()
    top = [i for i in range(len(g)) if tuple(g[i]) == (1, 2)]
    assert len(top) == 4, g
    np.testing.assert_allclose(dist[top], -1e-3, atol=1e-9)
    xs = sorted({round(p[0], 9) for p in pos[top]})
    np.testing.assert_allclose(xs, [-0.08, 0.1], atol=1e-9)  # the overlap spans x in [-0.08, 0.1]
    np.testing.assert_allclose(fr[top, :3], np.tile([0, 0, 1.0], (4, 1)), atol=1e-9)
