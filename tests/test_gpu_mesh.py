"""GPU parity of mesh geoms and the general convex narrow phase: contacts of
plane-mesh, plane-ellipsoid, plane-cylinder and MPR pairs (step.hip convex_convex / mpr_penetration
against oracle.c col_convex), rollouts of a scene that rests on them, rangefinders and depth / colour
renders that hit meshes (raymesh.h against oracle.c ray_mesh).  Pair lists are integer output and
bit-exact; geometry within fp32 tolerances stated per test.
"""
import numpy as np
import pytest

from mujoco_ros2_simulation_amd import sim, synth
import binding

pytestmark = pytest.mark.gpu

CUBE = "-1 -1 -1 1 -1 -1 -1 1 -1 1 1 -1 -1 -1 1 1 -1 1 -1 1 1 1 1 1"


def _rock(n=24, seed=3):
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(n, 3))
    v = v / np.linalg.norm(v, axis=1, keepdims=True) * rng.uniform(0.8, 1.0, size=(n, 1)) * [0.09, 0.07, 0.06]
    return " ".join(f"{x:.6f}" for x in v.ravel())


MESH_SCENE = f"""<mujoco><option timestep="0.002"/>
  <asset><mesh name="cube" vertex="{CUBE}" scale="0.06 0.06 0.06"/><mesh name="rock" vertex="{_rock()}"/></asset>
  <worldbody><geom type="plane" size="0 0 1"/>
    <body name="cube" pos="0 0 0.15" euler="10 20 30"><freejoint/><geom type="mesh" mesh="cube"/></body>
    <body name="rock" pos="0.25 0 0.15" euler="5 0 40"><freejoint/><geom type="mesh" mesh="rock"/></body>
    <body name="ell" pos="-0.25 0 0.15" euler="0 30 0"><freejoint/><geom type="ellipsoid" size="0.08 0.05 0.04"/></body>
    <body name="cyl" pos="0 0.25 0.15" euler="15 0 0"><freejoint/><geom type="cylinder" size="0.05 0.04"/></body>
    <body name="ball" pos="0.25 0.02 0.32"><freejoint/><geom type="sphere" size="0.04"/></body>
    <body name="box" pos="0.02 0.01 0.3" euler="0 0 20"><freejoint/><geom type="box" size="0.05 0.04 0.03"/></body>
  </worldbody></mujoco>"""


def _states(model, steps, n=8):
    b = sim.Batch(model, n)
    q0 = synth.initial_qpos(model, np.arange(n))
    b.set(sim.FIELD_QPOS, q0)
    b.step(steps)
    q = b.get(sim.FIELD_QPOS)
    b.close()
    return q


@pytest.mark.parametrize("steps", [100, 150, 300])
def test_mesh_convex_contact_lists(steps):
    """contacts after a forward pass from the same state: (geom1, geom2) lists bit-exact; dist within
    1e-4; normals within 2e-3 and positions within 2e-3 (MPR stops at the first portal within 1e-6 of
    the surface, and fp32 / fp64 can stop on neighbouring portals of a flat face: the depth agrees,
    the interpolated point moves along the face)"""
    model = sim.Model.from_string(MESH_SCENE)
    qs = _states(model, steps)
    b = sim.Batch(model, len(qs))
    b.set(sim.FIELD_QPOS, qs)
    b.forward()
    total, kinds = 0, set()
    for e, q in enumerate(qs):
        g, dist, pos, frame = b.contacts(e)
        d = binding.OracleData(model)
        d.qpos[:] = q
        d.forward()
        gr, dr, pr, fr = d.contacts()
        assert np.array_equal(g, gr), (e, g.tolist(), gr.tolist())
        np.testing.assert_allclose(dist, dr, atol=1e-4)
        np.testing.assert_allclose(frame[:, :3], fr[:, :3], atol=2e-3)
        np.testing.assert_allclose(pos, pr, atol=2e-3)
        total += len(g)
        kinds |= {tuple(model.geom_type[p]) for p in g}
    b.close()
    assert total >= 4 * len(qs)
    # plane-mesh, plane-ellipsoid and plane-cylinder in every state; the ball and the box land on the
    # meshes around steps 100-160 (sphere-mesh and box-mesh MPR pairs)
    assert {(0, 7), (0, 4), (0, 5)} <= kinds
    if steps <= 150:
        assert {(2, 7), (6, 7)} <= kinds


def test_mesh_scene_rollout():
    """200 steps of the mesh scene from the same start on both sides: qpos within 10x the scene's
    fp32-state sensitivity + 1e-5 (bodies settling on single-contact convex pairs).  The face contacts
    of polytope pairs are off here (RESTATE_NO_MULTICCD, both sides): the box landing on the cube gets
    clipped-polygon contacts whose vertices cross the zero-margin threshold as it settles, and fp32 /
    fp64 geometry switch such a contact on one step apart, so a free rollout measures that threshold,
    not the arithmetic (the face contacts' own tests: test_face_contacts_match_oracle,
    test_reseeded_face_contacts)"""
    model = sim.Model.from_string(MESH_SCENE)
    model.set_restate(sim.RESTATE_NO_MULTICCD)
    n, steps = 4, 200
    q0 = synth.initial_qpos(model, np.arange(n))
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, q0)
    b.step(steps)
    q = b.get(sim.FIELD_QPOS)
    b.close()
    ref, ref32 = np.zeros_like(q), np.zeros_like(q)
    for e in range(n):
        for out, rnd in ((ref, False), (ref32, True)):
            d = binding.OracleData(model)
            d.qpos[:] = q0[e]
            for _ in range(steps):
                d.step()
                if rnd:
                    d.qpos[:] = d.qpos.astype(np.float32)
                    d.qvel[:] = d.qvel.astype(np.float32)
            out[e] = d.qpos
    scale = np.maximum(np.abs(ref), 1.0)
    err = np.max(np.abs(q - ref) / scale)
    sens = np.max(np.abs(ref32 - ref) / scale)
    print(f"mesh scene 200 steps: qpos err {err:.2e}, fp32-state sensitivity {sens:.2e}")
    assert err <= 10 * sens + 1e-5
    # everything rests on the floor or on each other: no body fell through
    z = q[:, 2::7]
    assert np.all(z > 0.02)


def _site(i):
    """a ray in the fan: yaw -60..60 deg about +x, pitch 80..100 deg from +z"""
    yaw, pitch = np.radians(-60 + 2 * i), np.radians(80 + (i % 5) * 5)
    z = (np.cos(yaw) * np.sin(pitch), np.sin(yaw) * np.sin(pitch), np.cos(pitch))
    return f'<site name="s{i}" zaxis="{z[0]:.6f} {z[1]:.6f} {z[2]:.6f}"/>'


RAY_SCENE = f"""<mujoco><asset><mesh name="rock" vertex="{_rock(40, 7)}" scale="3 3 3"/></asset>
  <worldbody><geom type="plane" size="0 0 1"/>
    <body name="rock" pos="0.6 0 0.25" euler="10 20 30"><freejoint/><geom type="mesh" mesh="rock"/></body>
    <body name="spin" pos="0 0 0.25"><joint name="yaw" axis="0 0 1"/><geom type="cylinder" size="0.03 0.02" mass="1"/>
      {''.join(_site(i) for i in range(60))}</body>
  </worldbody>
  <sensor>{''.join(f'<rangefinder name="lidar-{i}" site="s{i}"/>' for i in range(60))}</sensor></mujoco>"""


def test_rangefinders_hit_mesh():
    """60 rangefinders sweeping a mesh rock (the lidar body spins): GPU sensordata equals the oracle's
    mj_rayMesh within 2e-5 * range on every ray that hits"""
    model = sim.Model.from_string(RAY_SCENE)
    n = 6
    q = np.tile(model.qpos0, (n, 1))
    q[:, 7] = np.linspace(-0.6, 0.6, n)
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, q)
    b.forward()
    sd = b.get(sim.FIELD_SENSORDATA)
    b.close()
    rock_hits = 0
    for e in range(n):
        d = binding.OracleData(model)
        d.qpos[:] = q[e]
        d.forward()
        ref = d.sensordata.copy()
        hit = ref >= 0
        assert np.array_equal(sd[e] >= 0, hit)
        np.testing.assert_allclose(sd[e][hit], ref[hit], rtol=2e-5, atol=2e-5)
        rock_hits += int(np.sum((ref > 0) & (ref < 0.9)))
    assert rock_hits > 20


def test_depth_rgb_with_mesh():
    """depth and colour of a frame with a mesh rock and a cube mesh against the oracle: depth within
    1e-5 on >= 99.9% of pixels, colour within 1 on >= 99%"""
    xml = f"""<mujoco><asset><mesh name="rock" vertex="{_rock(40, 7)}" scale="4 4 4"/>
      <mesh name="cube" vertex="{CUBE}" scale="0.2 0.2 0.2"/></asset><worldbody>
      <geom type="plane" size="0 0 1" rgba="0.5 0.5 0.5 1"/>
      <geom type="mesh" mesh="rock" pos="0.2 0.3 0.3" rgba="0.9 0.4 0.1 1"/>
      <geom type="mesh" mesh="cube" pos="-0.5 -0.2 0.2" euler="10 20 30" rgba="0.1 0.6 0.9 1"/>
      <camera name="cam" pos="0 -2 1.2" euler="63 0 0" fovy="60" resolution="320 240"/>
    </worldbody></mujoco>"""
    model = sim.Model.from_string(xml)
    b = sim.Batch(model, 2)
    b.forward()
    depth, rgb = b.render_rgbd(0, 0, 2)
    b.close()
    d = binding.OracleData(model)
    d.forward()
    wd, wrgb = d.render_rgbd(0)
    for e in range(2):
        assert np.isclose(depth[e], wd, rtol=1e-5, atol=1e-5).mean() >= 0.999
        diff = np.abs(rgb[e].astype(int) - wrgb.astype(int)).max(axis=-1)
        assert (diff <= 1).mean() >= 0.99
    # both meshes are in view: orange-dominant and blue-dominant regions
    assert np.sum(wrgb[..., 0] > wrgb[..., 2] + 30) > 500 and np.sum(wrgb[..., 2] > wrgb[..., 0] + 30) > 500


# ---------------------------------------------------------------- large meshes: the ray hierarchy
from pathlib import Path  # noqa: E402

ARM7_MESH = Path(__file__).resolve().parents[1] / "scenes" / "arm7_mesh.xml"


def _mesh_robot(resolution=None):
    xml = ARM7_MESH.read_text()
    if resolution:
        xml = xml.replace('resolution="640 480"', f'resolution="{resolution}"')
    return sim.Model.from_string(xml, str(ARM7_MESH.parent))


def _mesh_robot_states(model, n=8, steps=40):
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, synth.initial_qpos(model, np.arange(n)))
    b.set(sim.FIELD_CTRL, synth.ctrl_table(model, np.arange(n), 1, 10)[0])
    b.step(steps)
    q = b.get(sim.FIELD_QPOS)
    b.close()
    return q


def test_bvh_matches_every_triangle(monkeypatch):
    """the mesh robot (7 link shells of 1536 triangles, a 6912-triangle statue): rangefinders, depth and
    colour with the ray hierarchy equal the every-triangle traversal bit for bit (MRS_NO_BVH) -- the
    hierarchy only skips triangles whose inflated boxes the ray misses or enters past the nearest hit,
    and every triangle's t comes from the same ray_tri"""
    model = _mesh_robot("160 120")
    assert max(model.mesh_facenum) >= 5000
    q = _mesh_robot_states(model)
    out = []
    for flag in (None, "1"):
        if flag:
            monkeypatch.setenv("MRS_NO_BVH", flag)
        b = sim.Batch(model, len(q))
        b.set(sim.FIELD_QPOS, q)
        b.forward()
        depth, rgb = b.render_rgbd(0, 0, len(q))
        out.append((b.get(sim.FIELD_SENSORDATA), depth, rgb))
        b.close()
    (s1, d1, c1), (s2, d2, c2) = out
    assert np.array_equal(s1, s2)
    assert np.array_equal(d1, d2)
    assert (np.abs(c1.astype(int) - c2.astype(int)).max(axis=-1) == 0).mean() >= 0.999  # ties at shared edges


def test_rangefinders_mesh_robot():
    """C3's 360-beam lidar on the mesh robot: GPU sensordata against the oracle's brute-force
    mj_rayMesh within 2e-5 x range on >= 99.5% of rays, hit / miss identical on >= 99.8%, and the
    scan does see the link shells and the statue"""
    model = _mesh_robot()
    q = _mesh_robot_states(model)
    b = sim.Batch(model, len(q))
    b.set(sim.FIELD_QPOS, q)
    b.forward()
    sd = b.get(sim.FIELD_SENSORDATA)
    b.close()
    nrf = sum(1 for i in range(model.nsensor) if model.sensor_type[i] == sim.SENS_RANGEFINDER)
    close = same = total = mesh_hits = 0
    for e in range(len(q)):
        d = binding.OracleData(model)
        d.qpos[:] = q[e]
        d.forward()
        ref, got = d.sensordata[:nrf], sd[e, :nrf]
        hit = ref >= 0
        same += int(np.sum((got >= 0) == hit))
        close += int(np.sum(np.abs(got - ref) <= 2e-5 * np.maximum(np.abs(ref), 1)))
        total += nrf
        mesh_hits += int(np.sum((ref > 0.3) & (ref < 2.2)))  # arm shells / statue range band
    assert same >= 0.998 * total and close >= 0.995 * total, (same, close, total)
    assert mesh_hits > 100


def test_depth_mesh_robot():
    """a 160x120 depth + colour frame of the mesh robot against the oracle's per-pixel brute force:
    depth within 1e-5 on >= 99.9% of pixels, colour within 1 level on >= 99%"""
    model = _mesh_robot("160 120")
    q = _mesh_robot_states(model, n=2)
    b = sim.Batch(model, 2)
    b.set(sim.FIELD_QPOS, q)
    b.forward()
    depth, rgb = b.render_rgbd(0, 0, 2)
    b.close()
    for e in range(2):
        d = binding.OracleData(model)
        d.qpos[:] = q[e]
        d.forward()
        wd, wrgb = d.render_rgbd(0)
        assert np.isclose(depth[e], wd, rtol=1e-5, atol=1e-5).mean() >= 0.999
        diff = np.abs(rgb[e].astype(int) - wrgb.astype(int)).max(axis=-1)
        assert (diff <= 1).mean() >= 0.99


@pytest.mark.parametrize("resolution", ["640 480", "1280 720"])
def test_binned_frames_match_per_pixel_kernel(resolution, monkeypatch):
    """the triangle-binning frame kernel (depth_kernel_mesh, the default for scenes with mesh geoms)
    against the per-pixel hierarchy kernel (depth_kernel_v2, MRS_DEPTH_V2) on 8 states of the mesh robot
    at full resolution: depth bit-identical on >= 99.5% of pixels (both take the nearest ray_tri over the
    triangles whose boxes can contain the pixel, and the same primitive tests); the rest (~0.3%, the
    statue's folds seen edge-on) within 2e-4 of depth -- there t is ill-conditioned and the two kernels'
    fp32 rays land a few ulps apart, each as far from the fp64 oracle as the other (scripts/diag_mesh.py
    prints both against it) -- and colour identical except where two triangles are hit at exactly the
    same t (the shared edge of a mesh: either normal)."""
    model = _mesh_robot(resolution)
    q = _mesh_robot_states(model, n=8)
    out = {}
    for key in ("bin", "v2"):
        if key == "v2":
            monkeypatch.setenv("MRS_DEPTH_V2", "1")
        b = sim.Batch(model, 8)
        b.set(sim.FIELD_QPOS, q)
        b.forward()
        out[key] = b.render_rgbd(0, 0, 8)
        b.close()
    (db, cb), (dv, cv) = out["bin"], out["v2"]
    eq = db == dv
    print(f"{resolution}: depth bit-identical on {eq.mean():.6f} of pixels")
    assert eq.mean() >= 0.995
    assert np.max(np.abs(db - dv) / np.maximum(dv, 1)) <= 2e-4
    same = np.all(cb == cv, axis=-1)
    print(f"{resolution}: colour equal on {same.mean():.6f} of pixels")
    assert same.mean() >= 0.9995
    assert np.sum(db < db.max()) > 1000  # the meshes are in view


# ---------------------------------------------------------------- MPR pairs, re-seeded per step
MPR_SCENE = f"""<mujoco><option timestep="0.002" solver="PGS" iterations="50"/>
  <asset><mesh name="rock" vertex="{_rock(40, 7)}" scale="3 3 3"/></asset>
  <worldbody><geom type="plane" size="0 0 1"/>
    <geom name="rock" type="mesh" mesh="rock" pos="0 0 0.12" euler="10 20 30"/>
    <body name="e1" pos="0.02 0.01 0.36"><freejoint/><geom type="ellipsoid" size="0.06 0.05 0.04"/></body>
    <body name="e2" pos="-0.05 0.08 0.48"><freejoint/><geom type="ellipsoid" size="0.05 0.04 0.05"/></body>
    <body name="s1" pos="0.1 -0.06 0.42"><freejoint/><geom type="sphere" size="0.04"/></body>
    <body name="c1" pos="-0.12 -0.08 0.40"><freejoint/><geom type="capsule" size="0.03 0.04"/></body>
  </worldbody></mujoco>"""


def test_reseeded_mpr_pairs():
    """one step at a time from the oracle's state (test_gpu_solvers._reseeded): bodies with curved
    surfaces (ellipsoids, a sphere, a capsule) tumbling over a static mesh rock and each other, so the
    contacts are MPR pairs (ellipsoid-mesh, sphere-mesh, capsule-mesh, ellipsoid-ellipsoid).  Contact
    pairs agree (flips explained as threshold cases) and the per-step state within 1e-5: MPR's normal
    is refined on both sides by the polish (the minimiser of the Minkowski support
    function next to MPR's portal, which MPR alone fixes only to ~sqrt(2 tol / r), 7e-3 rad), and the
    portal's nearest point is taken from its plane when the origin projects inside it (the barycentric
    formula cancels in fp32 on long thin portals: measured before, qpos 2e-4 / qvel 9e-2)"""
    from test_gpu_solvers import _reseeded
    model = sim.Model.from_string(MPR_SCENE)
    settle, steps = 75, 100
    d = binding.OracleData(model)
    d.qpos[:] = synth.initial_qpos(model, np.arange(1))[0]
    kinds = set()
    for t in range(settle + steps):
        d.step()
        if t >= settle:
            kinds |= {tuple(int(model.geom_type[x]) for x in p) for p in d.contacts()[0]}
    assert {(4, 7), (2, 7)} <= kinds, kinds  # ellipsoid-mesh and sphere-mesh MPR pairs occur
    wq, wv, ncon, flips, unexplained = _reseeded(model, 16, steps, settle=settle)
    print(f"MPR scene: worst per-step rel err qpos {wq:.2e} qvel {wv:.2e}; contacts {ncon.mean():.2f}; "
          f"flips {flips}; pair kinds {sorted(kinds)}")
    assert ncon.max() > 0
    assert flips <= max(1, 0.01 * 16 * steps)
    assert not unexplained, unexplained[:5]
    assert wq <= 1e-5 and wv <= 1e-5


# ---------------------------------------------------------------- many ray geoms (mesh slots, > 32 geoms)
def _ring_scene(n_mesh, n_small, static, nray=30):
    """a lidar of `nray` rays (every third pitched 4 deg down onto the floor) inside a ring of
    `n_mesh` mesh rocks at radius 1 and `n_small` spheres / boxes at radius 1.8; the lidar sits on a
    spinning body, or in the world (the static ray split)"""
    assets = "".join(f'<mesh name="r{k}" vertex="{_rock(30, 11 + k)}" scale="3 3 3"/>' for k in range(n_mesh))
    rocks = "".join(
        f'<geom type="mesh" mesh="r{k}" pos="{np.cos(2 * np.pi * k / n_mesh):.5f} {np.sin(2 * np.pi * k / n_mesh):.5f} 0.3" '
        f'euler="{7 * k} {11 * k} {13 * k}"/>' for k in range(n_mesh))
    smalls = ""
    for k in range(n_small):
        a = 2 * np.pi * (k + 0.5) / max(n_small, 1)
        pos = f'{1.8 * np.cos(a):.5f} {1.8 * np.sin(a):.5f} 0.3'
        smalls += (f'<geom type="sphere" size="0.09" pos="{pos}"/>' if k % 2 else
                   f'<geom type="box" size="0.07 0.08 0.09" pos="{pos}" euler="0 0 {17 * k}"/>')
    sites = ""
    for i in range(nray):
        a, p = 2 * np.pi * i / nray + 0.013, np.radians(94.0 if i % 3 == 0 else 90.3)
        z = (np.cos(a) * np.sin(p), np.sin(a) * np.sin(p), np.cos(p))
        sites += f'<site name="s{i}" zaxis="{z[0]:.6f} {z[1]:.6f} {z[2]:.6f}"/>'
    lidar = (f'<body name="post" pos="0 0 0.3">{sites}</body>' if static else
             f'<body name="spin" pos="0 0 0.3"><joint name="yaw" axis="0 0 1"/>'
             f'<geom type="cylinder" size="0.03 0.02" mass="1"/>{sites}</body>')
    sens = "".join(f'<rangefinder name="lidar-{i}" site="s{i}"/>' for i in range(nray))
    return (f'<mujoco><asset>{assets}</asset><worldbody><geom type="plane" size="0 0 1"/>{rocks}{smalls}'
            f'{lidar}</worldbody><sensor>{sens}</sensor></mujoco>')


@pytest.mark.parametrize("n_mesh,n_small,static", [(14, 0, False), (14, 0, True), (14, 24, False), (6, 40, True)])
def test_rangefinders_many_ray_geoms(n_mesh, n_small, static):
    """more mesh ray geoms than a 64-bit slot table of 5-bit indices can name (14 meshes with 2 rays
    per lane: 32 slots) and more than 32 ray geoms in all (the ray pass in chunks of 32): GPU
    sensordata equals the oracle's brute-force mj_ray within 2e-5 x range, hit / miss identical, and
    the rock ring is what most rays see"""
    model = sim.Model.from_string(_ring_scene(n_mesh, n_small, static))
    nrg = sum(1 for g in range(model.ngeom) if model.geom_rgba[g, 3] > 0)
    assert (nrg > 32) == (n_small > 0)
    n = 1 if static else 6
    q = np.tile(model.qpos0, (n, 1))
    if not static:
        q[:, 0] = np.linspace(-0.4, 0.4, n)
    b = sim.Batch(model, n)
    b.set(sim.FIELD_QPOS, q)
    b.forward()
    sd = b.get(sim.FIELD_SENSORDATA)
    b.close()
    for e in range(n):
        d = binding.OracleData(model)
        d.qpos[:] = q[e]
        d.forward()
        ref = d.sensordata.copy()
        hit = ref >= 0
        assert np.array_equal(sd[e] >= 0, hit), e
        np.testing.assert_allclose(sd[e][hit], ref[hit], rtol=2e-5, atol=2e-5)
        assert np.sum((ref > 0.6) & (ref < 1.2)) >= n_mesh  # rays end on the rock ring


def test_binned_frames_in_chunks(monkeypatch):
    """the binned kernel's per-frame triangle lists under a small memory budget (MRS_RAST_BUDGET_MB=1:
    frames rendered in several launches over a reused list) give the same frames bit for bit"""
    model = _mesh_robot("160 120")
    q = _mesh_robot_states(model, n=8)
    out = []
    for budget in (None, "1"):
        if budget:
            monkeypatch.setenv("MRS_RAST_BUDGET_MB", budget)
        b = sim.Batch(model, 8)
        b.set(sim.FIELD_QPOS, q)
        b.forward()
        out.append(b.render_rgbd(0, 0, 8))
        b.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])


LIT_SCENE = f"""<mujoco><visual><headlight ambient="0.05 0.05 0.05" diffuse="0.3 0.3 0.3" specular="0.2 0.2 0.2"/></visual>
  <asset><mesh name="rock" vertex="{_rock(40, 7)}" scale="4 4 4"/>
    <mesh name="cube" vertex="{CUBE}" scale="0.2 0.2 0.2"/>
    <texture type="skybox" builtin="gradient" rgb1="0.3 0.5 0.7" rgb2="0 0 0" width="64" height="384"/>
    <texture name="grid" type="2d" builtin="checker" mark="edge" rgb1="0.2 0.3 0.4" rgb2="0.1 0.2 0.3"
             markrgb="0.8 0.8 0.8" width="300" height="300"/>
    <material name="floor" texture="grid" texuniform="true" texrepeat="5 5" reflectance="0.2"/>
    <material name="shiny" specular="0.9" shininess="0.8" emission="0.1" rgba="0.8 0.2 0.2 1"/></asset>
  <worldbody>
    <light directional="true" pos="0 0 3" dir="0.3 0.2 -1" castshadow="true"/>
    <light pos="1 -1 2" dir="-0.5 0.5 -1" cutoff="50" exponent="5" attenuation="1 0.1 0.02"
           diffuse="0.5 0.4 0.3" specular="0.4 0.4 0.4" castshadow="true"/>
    <geom type="plane" size="0 0 1" material="floor"/>
    <geom type="mesh" mesh="rock" pos="0.2 0.3 0.3" rgba="0.9 0.4 0.1 1"/>
    <geom type="mesh" mesh="cube" pos="-0.5 -0.2 0.2" euler="10 20 30" rgba="0.1 0.6 0.9 1"/>
    <geom type="sphere" size="0.15" pos="0.5 -0.4 0.4" material="shiny"/>
    <geom type="capsule" size="0.06 0.2" pos="-0.3 0.5 0.5" euler="30 40 0" rgba="0.2 0.9 0.3 1"/>
    <geom type="box" size="0.1 0.15 0.05" pos="0.1 -0.7 0.6" euler="10 0 25" rgba="0.9 0.9 0.2 1"/>
    <camera name="cam" pos="0 -2.2 1.0" euler="72 0 0" fovy="70" resolution="320 240"/>
  </worldbody></mujoco>"""


@pytest.mark.parametrize("path", ["raster", "v2", "tile"])
def test_lit_colour_all_kernels(path, monkeypatch):
    """the lit colour model (lit.h lit_pixel against oracle.c lit_color): headlight, a directional and
    a spot light (both castshadow), a checker-textured floor with edge marks, a specular emissive
    material and the gradient skybox, rendered by each frame kernel -- the mesh binning kernel
    (default), depth_kernel_v2 (MRS_DEPTH_V2) and the tile kernel (MRS_DEPTH_V1).  Depth within 1e-5
    on >= 99.9% of pixels; colour within 1 level on >= 98% (fp32 against fp64 moves silhouettes,
    shadow edges, texel and spot-cone boundaries by a pixel); shadows, texture and sky are present."""
    if path == "v2":
        monkeypatch.setenv("MRS_DEPTH_V2", "1")
    elif path == "tile":
        monkeypatch.setenv("MRS_DEPTH_V1", "1")
    model = sim.Model.from_string(LIT_SCENE)
    b = sim.Batch(model, 2)
    b.forward()
    depth, rgb = b.render_rgbd(0, 0, 2)
    np.testing.assert_array_equal(depth, b.render_depth(0, 0, 2))
    b.close()
    d = binding.OracleData(model)
    d.forward()
    wd, wrgb = d.render_rgbd(0)
    for e in range(2):
        assert np.isclose(depth[e], wd, rtol=1e-5, atol=1e-5).mean() >= 0.999
        diff = np.abs(rgb[e].astype(int) - wrgb.astype(int)).max(axis=-1)
        assert (diff <= 1).mean() >= 0.98, (diff <= 1).mean()
    miss = wd >= wd.max()
    assert miss.sum() > 1000 and wrgb[miss][:, 2].max() > 100  # skybox above the horizon
    assert len({tuple(c) for c in wrgb.reshape(-1, 3)[::37]}) > 100


# ---------------------------------------------------------------- polytope face contacts (multiccd)
_CUBE = 'vertex="-1 -1 -1 1 -1 -1 1 1 -1 -1 1 -1 -1 -1 1 1 -1 1 1 1 1 -1 1 1" scale="0.08 0.08 0.08"'
FACE_SCENE = f"""<mujoco><compiler angle="radian"/><option timestep="0.002" solver="PGS" iterations="50"/>
  <asset><mesh name="cube" {_CUBE}/></asset>
  <worldbody><geom name="table" type="box" pos="0 0 -0.05" size="1 1 0.05"/>
    <body name="a" pos="0.3 0.1 0.09" euler="0.02 -0.03 0.2"><freejoint/><geom type="mesh" mesh="cube"/></body>
    <body name="b" pos="-0.25 -0.2 0.12" euler="0.1 0.05 -0.4"><freejoint/><geom type="mesh" mesh="cube"/></body>
    <body name="c" pos="0 0.35 0.085"><freejoint/><geom type="mesh" mesh="cube"/></body>
    <body name="d" pos="0.03 0.36 0.26" euler="0 0 0.5"><freejoint/><geom type="mesh" mesh="cube"/></body>
    <body name="e" pos="-0.3 0.3 0.2"><freejoint/><geom type="box" size="0.06 0.05 0.04" euler="0.05 0 0.3"/></body>
  </worldbody></mujoco>"""


def _face_kinds(model, d):
    return {tuple(int(model.geom_type[x]) for x in p) for p in d.contacts()[0]}


def test_face_contacts_match_oracle():
    """mesh cubes resting on a box table, a cube stacked on another (mesh-mesh) and a box (box-mesh):
    the face contacts of polytope pairs (up to one per clipped polygon vertex) agree with the oracle --
    the (geom1, geom2) list bit-exact, dist / pos / frame within 1e-4 -- after the cubes have settled"""
    model = sim.Model.from_string(FACE_SCENE)
    d = binding.OracleData(model)
    d.step(300)
    q = d.qpos.copy()
    g_ref = d.contacts()[0]
    per_pair = {}
    for p in g_ref.tolist():
        per_pair[tuple(p)] = per_pair.get(tuple(p), 0) + 1
    assert max(per_pair.values()) >= 4, per_pair  # flat rests give several contacts per pair
    assert (6, 7) in _face_kinds(model, d) and (7, 7) in _face_kinds(model, d)
    b = sim.Batch(model, 4)
    b.set(sim.FIELD_QPOS, np.tile(q, (4, 1)))
    b.forward()
    for e in range(4):
        g, dist, pos, frame = b.contacts(e)
        r = binding.OracleData(model)
        r.qpos[:] = q
        r.forward()
        gr, dr, pr, fr = r.contacts()
        assert np.array_equal(g, gr), (g.tolist(), gr.tolist())
        np.testing.assert_allclose(dist, dr, atol=1e-4)
        np.testing.assert_allclose(pos, pr, atol=1e-4)
        np.testing.assert_allclose(frame, fr, atol=1e-4)
    b.close()


def test_reseeded_face_contacts():
    """the same scene one step at a time from the oracle's state (test_gpu_solvers._reseeded) while
    the cubes fall, tip and settle: per-step qpos / qvel within 1e-5, contact-count flips explained as
    threshold cases"""
    from test_gpu_solvers import _reseeded
    model = sim.Model.from_string(FACE_SCENE)
    wq, wv, ncon, flips, unexplained = _reseeded(model, 8, 120, settle=40)
    print(f"face-contact scene: worst per-step rel err qpos {wq:.2e} qvel {wv:.2e}; contacts {ncon.mean():.2f}; "
          f"flips {flips}")
    assert ncon.max() >= 12
    assert flips <= max(1, 0.01 * 8 * 120)
    assert not unexplained, unexplained[:5]
    assert wq <= 1e-5 and wv <= 1e-5
