"""Mesh geoms and the general convex narrow phase on the CPU: the compiler's mesh
processing (csrc/mjcf/mesh.cc, compiler.cc parse_asset) pinned by closed-form answers, and the
oracle's mesh ray cast / plane-mesh / MPR contacts (oracle.c ray_mesh, col_plane_mesh, col_convex)
against the analytic primitives they must reproduce.  MuJoCo's own mesh compiler and libccd are
third-party and absent here: these are first-principles known answers, not reference vectors.
"""
import struct

import numpy as np
import pytest

from mujoco_ros2_simulation_amd import sim
import binding

CUBE = "-1 -1 -1 1 -1 -1 -1 1 -1 1 1 -1 -1 -1 1 1 -1 1 -1 1 1 1 1 1"


def scene(assets, bodies, floor=True):
    return sim.Model.from_string(f"""<mujoco><asset>{assets}</asset><worldbody>
      {'<geom type="plane" size="0 0 1"/>' if floor else ''}{bodies}</worldbody></mujoco>""")


def test_cube_mesh_inertia_equals_box():
    """a cube given by its 8 corners plus interior points, scaled (0.05, 0.1, 0.2): box mass and
    inertia, hull of the 8 corners, bounding box = half sizes"""
    m = scene(f'<mesh name="c" vertex="{CUBE} 0 0 0 0.5 0.5 0.5" scale="0.05 0.1 0.2"/>',
              '<body><freejoint/><geom type="mesh" mesh="c"/></body>', floor=False)
    mass = 1000 * 0.1 * 0.2 * 0.4
    assert m.nmesh == 1 and m.mesh_hullnum[0] == 8 and m.mesh_vertnum[0] == 10
    assert m.body_mass[1] == pytest.approx(mass)
    I = mass * np.array([0.2 ** 2 + 0.4 ** 2, 0.1 ** 2 + 0.4 ** 2, 0.1 ** 2 + 0.2 ** 2]) / 12
    np.testing.assert_allclose(np.sort(m.body_inertia[1]), np.sort(I), rtol=1e-10)
    np.testing.assert_allclose(np.sort(m.geom_size[0]), [0.05, 0.1, 0.2], rtol=1e-10)
    assert m.geom_rbound[0] == pytest.approx(np.sqrt(0.05 ** 2 + 0.1 ** 2 + 0.2 ** 2))


def test_tetrahedron_recentred_at_com():
    """right tetrahedron of leg a at the origin: volume a^3/6, centre of mass (a/4, a/4, a/4); the geom
    frame moves to the centre of mass (MuJoCo's mesh frame) and the vertices are re-expressed in it"""
    a = 0.3
    m = scene(f'<mesh name="t" vertex="0 0 0 {a} 0 0 0 {a} 0 0 0 {a}"/>',
              '<body pos="1 2 3"><freejoint/><geom type="mesh" mesh="t" pos="0.1 0 0"/></body>', floor=False)
    assert m.body_mass[1] == pytest.approx(1000 * a ** 3 / 6)
    np.testing.assert_allclose(m.geom_pos[0], [0.1 + a / 4, a / 4, a / 4], atol=1e-12)
    v = m.mesh_vert
    np.testing.assert_allclose(v.mean(axis=0), 0, atol=1e-12)  # vertex centroid = volume centroid here
    # the world-frame corners are unchanged by the recentring
    w, x, y, z = m.geom_quat[0]
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    corners = v @ R.T + m.geom_pos[0]
    want = np.array([[0, 0, 0], [a, 0, 0], [0, a, 0], [0, 0, a]]) + [0.1, 0, 0]
    for c in want:
        assert np.min(np.linalg.norm(corners - c, axis=1)) < 1e-12


def _write_obj(path, verts, faces):
    with open(path, "w") as f:
        for v in verts:
            f.write("v %r %r %r\n" % tuple(map(float, v)))
        for t in faces:
            f.write("f " + " ".join(f"{i + 1}/1" for i in t) + "\n")


def _cube_faces():
    # outward quads of the CUBE corner order (bit 0: x, bit 1: y, bit 2: z)
    return [(0, 2, 3, 1), (4, 5, 7, 6), (0, 1, 5, 4), (2, 6, 7, 3), (0, 4, 6, 2), (1, 3, 7, 5)]


def test_obj_and_stl_files(tmp_path):
    """the same cube from an OBJ file (quads fanned), a binary STL and an ASCII STL (vertices merged),
    found through <compiler meshdir>; equal mass properties"""
    verts = np.array(CUBE.split(), dtype=float).reshape(8, 3) * 0.1
    (tmp_path / "meshes").mkdir()
    _write_obj(tmp_path / "meshes" / "cube.obj", verts, _cube_faces())
    tris = [(q[0], q[k], q[k + 1]) for q in _cube_faces() for k in (1, 2)]
    with open(tmp_path / "meshes" / "cube.stl", "wb") as f:
        f.write(b"\0" * 80 + struct.pack("<I", len(tris)))
        for t in tris:
            f.write(struct.pack("<3f", 0, 0, 0) + b"".join(struct.pack("<3f", *verts[i]) for i in t) + b"\0\0")
    with open(tmp_path / "meshes" / "cube_ascii.stl", "w") as f:
        f.write("solid c\n")
        for t in tris:
            f.write("facet normal 0 0 0\nouter loop\n" + "".join("vertex %r %r %r\n" % tuple(map(float, verts[i])) for i in t)
                    + "endloop\nendfacet\n")
        f.write("endsolid c\n")
    for fname in ("cube.obj", "cube.stl", "cube_ascii.stl"):
        xml = f"""<mujoco><compiler meshdir="meshes"/><asset><mesh file="{fname}"/></asset><worldbody>
          <body><freejoint/><geom type="mesh" mesh="{fname.split('.')[0]}"/></body></worldbody></mujoco>"""
        m = sim.Model.from_string(xml, str(tmp_path))
        assert m.mesh_vertnum[0] == 8 and m.mesh_facenum[0] == 12, fname
        assert m.body_mass[1] == pytest.approx(1000 * 0.2 ** 3), fname
        np.testing.assert_allclose(m.body_inertia[1], 1000 * 0.2 ** 3 * 2 * 0.1 ** 2 / 3, rtol=1e-6)


@pytest.mark.parametrize("bad, msg", [('vertex="0 0 0 1 0 0 0 1 0 1 1 0"', "coplanar"),
                                      ('vertex="0 0 0 1 0 0"', "at least 4"),
                                      ('file="missing.obj"', "cannot open")])
def test_bad_meshes_are_errors(bad, msg):
    with pytest.raises(sim.MrsError, match=msg):
        scene(f'<mesh name="x" {bad}/>', '<body><freejoint/><geom type="mesh" mesh="x"/></body>')


def test_mesh_ray_equals_box_ray():
    """rays onto a cube mesh and onto the same box (rotated body) hit at the same distance"""
    m = scene(f'<mesh name="c" vertex="{CUBE}" scale="0.1 0.2 0.3"/>',
              '<body euler="20 30 40"><geom type="mesh" mesh="c"/></body>'
              '<body pos="3 0 0" euler="20 30 40"><geom type="box" size="0.1 0.2 0.3"/></body>', floor=False)
    d = binding.OracleData(m)
    d.forward()
    rng = np.random.default_rng(0)
    hits = 0
    for _ in range(200):
        p = rng.normal(size=3) * 0.1 + [0, 0, 1.5]
        v = -p + rng.normal(size=3) * 0.15
        t1, g1 = d.ray(p, v, -1)
        t2, g2 = d.ray(p + [3, 0, 0], v, -1)
        assert (g1 < 0) == (g2 < 0)
        if g1 >= 0:
            hits += 1
            assert t1 == pytest.approx(t2, rel=1e-9, abs=1e-12)
    assert hits > 50


def test_mesh_cube_rests_like_box_and_convex_primitives_settle():
    """a cube mesh on the floor settles exactly like the box (plane-mesh gives the 4 bottom corners);
    an ellipsoid (one support contact) and an upright cylinder (3 rim contacts) rest at their size"""
    m = scene(f'<mesh name="c" vertex="{CUBE}" scale="0.1 0.1 0.1"/>',
              '<body pos="0 0 0.3"><freejoint/><geom type="mesh" mesh="c"/></body>'
              '<body pos="0.5 0 0.3"><freejoint/><geom type="box" size="0.1 0.1 0.1"/></body>'
              '<body pos="-0.5 0 0.3"><freejoint/><geom type="ellipsoid" size="0.1 0.15 0.1"/></body>'
              '<body pos="-1 0 0.3"><freejoint/><geom type="cylinder" size="0.1 0.1"/></body>')
    d = binding.OracleData(m)
    for _ in range(800):
        d.step()
    q = d.qpos.reshape(4, 7)
    np.testing.assert_allclose(q[0, :3] - [0, 0, 0], q[1, :3] - [0.5, 0, 0], atol=1e-15)
    np.testing.assert_allclose(q[:, 2], 0.1, atol=1e-3)
    assert d.ncon == 4 + 4 + 1 + 3


def _pair(g1, g2, p2, margin=0.0, restate=0):
    m = sim.Model.from_string(f"""<mujoco><asset><mesh name="c" vertex="{CUBE}" scale="0.1 0.1 0.1"/></asset>
      <worldbody><body><freejoint/>{g1}</body><body pos="{p2}"><freejoint/>{g2}</body></worldbody></mujoco>"""
                              .replace("<geom ", f'<geom margin="{margin}" '))
    m.set_restate(restate)
    d = binding.OracleData(m)
    d.forward()
    return d.contacts()


def test_mpr_sphere_ellipsoid_is_exact():
    """MPR on a sphere and a round ellipsoid converges to the analytic sphere-sphere contact"""
    c = np.array([0.15, 0.05, 0.02])
    g, dist, pos, frame = _pair('<geom type="sphere" size="0.1"/>', '<geom type="ellipsoid" size="0.1 0.1 0.1"/>',
                                " ".join(map(str, c)))
    assert len(dist) == 1
    assert dist[0] == pytest.approx(np.linalg.norm(c) - 0.2, abs=1e-9)
    np.testing.assert_allclose(frame[0, :3], c / np.linalg.norm(c), atol=1e-7)


@pytest.mark.parametrize("margin", [0.0, 0.02])
def test_mpr_box_mesh_face_depth(margin):
    """box vs cube mesh, face on face with an offset: MPR's depth along z as the SAT box-box gives; a
    margin inflates both shapes by margin/2 and is subtracted back (dist = margin - depth).  With the
    face contacts (default) the pair gives the four corners of the faces' overlap at that depth"""
    g, dist, pos, frame = _pair('<geom type="box" size="0.1 0.1 0.1"/>', '<geom type="mesh" mesh="c"/>',
                                "0.03 0.02 0.19", margin)
    assert len(dist) == 4
    np.testing.assert_allclose(dist, -0.01, atol=1e-9)
    np.testing.assert_allclose(frame[:, :3], np.tile([0, 0, 1.0], (4, 1)), atol=1e-9)
    np.testing.assert_allclose(sorted({round(p[0], 9) for p in pos}), [-0.07, 0.1], atol=1e-9)
    np.testing.assert_allclose(sorted({round(p[1], 9) for p in pos}), [-0.08, 0.1], atol=1e-9)
    g, dist, pos, frame = _pair('<geom type="box" size="0.1 0.1 0.1"/>', '<geom type="mesh" mesh="c"/>',
                                "0.03 0.02 0.19", margin, restate=sim.RESTATE_NO_MULTICCD)
    assert len(dist) == 1
    # margin rounds the inflated shapes' edges: MPR stops within mpr_tolerance (1e-6) of the surface
    assert dist[0] == pytest.approx(-0.01, abs=1e-9 if margin == 0 else 1e-6)
    np.testing.assert_allclose(frame[0, :3], [0, 0, 1], atol=1e-9 if margin == 0 else 1e-6)


def test_mpr_capsule_cylinder_side():
    """capsule (r 0.05) beside a cylinder (r 0.1), axes parallel, centres 0.12 apart: depth 0.03 along x"""
    g, dist, pos, frame = _pair('<geom type="capsule" size="0.05 0.1"/>', '<geom type="cylinder" size="0.1 0.1"/>',
                                "0.12 0 0", 0.01)
    assert dist[0] == pytest.approx(0.12 - 0.15, abs=1e-9)
    np.testing.assert_allclose(frame[0, :3], [1, 0, 0], atol=1e-9)


def test_mpr_separated_gives_no_contact():
    g, dist, pos, frame = _pair('<geom type="sphere" size="0.1"/>', '<geom type="mesh" mesh="c"/>', "0.25 0 0")
    assert len(dist) == 0
    g, dist, pos, frame = _pair('<geom type="sphere" size="0.1"/>', '<geom type="mesh" mesh="c"/>', "0.25 0 0", 0.06)
    assert len(dist) == 1 and dist[0] == pytest.approx(0.05, abs=1e-9)
