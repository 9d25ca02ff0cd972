"""Compiler known-answer tests for the benchmark scenes C3 (scenes/arm7_lidar.xml), C4
(scenes/mobile_base.xml) and C5 (scenes/arm_boxes.xml), derived here independently of the MJCF
compiler (csrc/mjcf/compiler.cc) -- the oracle steps the compiler's output, so a compiler error would
shift oracle and GPU alike; these pin the compiled constants to first principles:

* geom-derived body inertia: mass, centre of mass and the inertia tensor of every capsule link by
  numeric integration over thin slices of the solid (not the closed form the compiler uses), and of
  boxes / spheres by their textbook formulas;
* dof_M0 (diagonal of M at qpos0) by summing m |a x (c - p)|^2 + a' I a over each dof's subtree from
  the XML's body offsets and axes, and dampratio -> kv = 2 dampratio sqrt(kp M0) [upstream set0];
* the statically admissible collision pairs (mj_collision's broad-phase filters) counted from the
  scene's contype/conaffinity classes and body tree by hand, and listed identically by the compiler
  and by the oracle's own filter.
"""
from pathlib import Path

import numpy as np
import pytest

from conftest import ARM7
from mujoco_ros2_simulation_amd import sim
import binding

SCENES = ARM7.parent
RHO = 1000.0  # MJCF default geom density

# the C3/C5 arm: link k at height z_k above its parent, capsule fromto (0,0,0)-(0,0,L_k) radius r_k,
# hinge axes alternating z / y (scenes/arm7_lidar.xml, scenes/arm_boxes.xml)
ARM_OFFSETS = [0.3, 0.3, 0.3, 0.25, 0.25, 0.2, 0.15]   # body pos z of link1..link7 (link1 from base at 0)
ARM_LENGTHS = [0.3, 0.3, 0.25, 0.25, 0.2, 0.15, 0.1]
ARM_RADII = [0.06, 0.055, 0.05, 0.045, 0.04, 0.035, 0.03]
ARM_AXES = [(0, 0, 1), (0, 1, 0)] * 3 + [(0, 0, 1)]


def capsule_by_slices(r, L, n=40000):
    """mass, com z, Ixx (= Iyy) and Izz about the com of a density-RHO capsule whose axis runs from
    z = 0 to z = L, by integrating thin discs of radius rho(z) over z in [-r, L + r] (midpoint rule)"""
    z = -r + (np.arange(n) + 0.5) * (L + 2 * r) / n
    dz = (L + 2 * r) / n
    rho2 = np.where(z < 0, r * r - z * z, np.where(z > L, r * r - (z - L) ** 2, r * r))
    rho2 = np.maximum(rho2, 0)
    dm = RHO * np.pi * rho2 * dz
    mass = dm.sum()
    zc = (dm * z).sum() / mass
    izz = (0.5 * dm * rho2).sum()
    ixx = (dm * (rho2 / 4 + (z - zc) ** 2)).sum()
    return mass, zc, ixx, izz


def body_tensor(m, b):
    """inertia tensor of body b about its com, in the body frame: R(iquat) diag(I) R'"""
    w, x, y, z = m.body_iquat[b]
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                  [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                  [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
    return R @ np.diag(m.body_inertia[b]) @ R.T


def arm_expected():
    """per link: mass, com (world, qpos0), inertia tensor (world = body frame at qpos0); joint anchors"""
    links, z = [], 0.0
    for off, L, r in zip(ARM_OFFSETS, ARM_LENGTHS, ARM_RADII):
        z += off
        mass, zc, ixx, izz = capsule_by_slices(r, L)
        links.append((mass, np.array([0, 0, z + zc]), np.diag([ixx, ixx, izz]), np.array([0, 0, z])))
    return links


def arm_M0(links, armature=0.02):
    M0 = []
    for j, (_, _, _, p) in enumerate(links):
        a = np.array(ARM_AXES[j], dtype=float)
        v = armature
        for mass, c, I, _ in links[j:]:
            v += mass * np.dot(np.cross(a, c - p), np.cross(a, c - p)) + a @ I @ a
        M0.append(v)
    return np.array(M0)


@pytest.mark.parametrize("scene", ["arm7_lidar", "arm_boxes"])
def test_arm_links_inertia_by_integration(scene):
    m = sim.Model.load(SCENES / f"{scene}.xml")
    for k, (mass, com, I, anchor) in enumerate(arm_expected()):
        b = m.name2id(sim.OBJ_BODY, f"link{k + 1}")
        assert m.body_mass[b] == pytest.approx(mass, rel=1e-6)
        np.testing.assert_allclose(m.body_ipos[b], [0, 0, com[2] - anchor[2]], atol=1e-7)
        np.testing.assert_allclose(body_tensor(m, b), I, rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("scene", ["arm7_lidar", "arm_boxes"])
def test_arm_dof_M0_and_dampratio_kv(scene):
    m = sim.Model.load(SCENES / f"{scene}.xml")
    M0 = arm_M0(arm_expected())
    np.testing.assert_allclose(m.dof_M0[:7], M0, rtol=1e-6)
    # <position kp="1000" dampratio="1"/>: kv = 2 * 1 * sqrt(kp * M0) (gear 1), bias = -kv qvel
    np.testing.assert_allclose(-m.actuator_biasprm[:7, 2], 2 * np.sqrt(1000 * M0), rtol=1e-6)
    np.testing.assert_allclose(-m.actuator_biasprm[:7, 1], 1000)


def test_c5_boxes_inertia_and_free_dofs():
    """eight 0.1 m cubes of 0.3 kg: I = m (a^2 + b^2) / 3 with half sizes 0.05; a free joint's dofs
    carry (m, m, m, I, I, I) on the diagonal of M at qpos0 (no armature: <freejoint> takes no joint
    defaults); the boxes' stack partners start at the MJCF euler yaws"""
    m = sim.Model.load(SCENES / "arm_boxes.xml")
    I = 0.3 * (0.05 ** 2 + 0.05 ** 2) / 3
    for k in range(8):
        b = m.name2id(sim.OBJ_BODY, f"box{k + 1}")
        assert m.body_mass[b] == pytest.approx(0.3)
        np.testing.assert_allclose(body_tensor(m, b), np.eye(3) * I, rtol=1e-9, atol=1e-15)
        d = m.body_dofadr[b]
        np.testing.assert_allclose(m.dof_M0[d:d + 6], [0.3] * 3 + [I] * 3, rtol=1e-9)
    b5 = m.name2id(sim.OBJ_BODY, "box5")
    np.testing.assert_allclose(m.body_quat[b5], [np.cos(0.25), 0, 0, np.sin(0.25)], atol=1e-12)


def test_c4_base_inertia_and_M0():
    """mobile base: chassis box 8 kg (0.25, 0.18, 0.05), caster sphere 0.2 kg r 0.04 at (-0.2, 0,
    -0.06), wheels 0.5 kg spheres r 0.1 on their own hinge bodies at (0.1, +-0.22, 0); wheel dof M0 =
    2/5 m r^2 about the y axis through the sphere centre"""
    m = sim.Model.load(SCENES / "mobile_base.xml")
    base = m.name2id(sim.OBJ_BODY, "base")
    mass = 8 + 0.2
    assert m.body_mass[base] == pytest.approx(mass)
    com = np.array([-0.2 * 0.2, 0, -0.06 * 0.2]) / mass
    np.testing.assert_allclose(m.body_ipos[base], com, atol=1e-12)
    def shifted(mass_i, pos_i, I_i):        # parallel-axis theorem to the body com
        d = np.asarray(pos_i) - com
        return I_i + mass_i * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    chassis = np.diag([8 * (0.18 ** 2 + 0.05 ** 2) / 3, 8 * (0.25 ** 2 + 0.05 ** 2) / 3, 8 * (0.25 ** 2 + 0.18 ** 2) / 3])
    caster = np.eye(3) * 0.4 * 0.2 * 0.04 ** 2
    want = shifted(8.0, [0, 0, 0], chassis) + shifted(0.2, [-0.2, 0, -0.06], caster)
    np.testing.assert_allclose(body_tensor(m, base), want, rtol=1e-9, atol=1e-12)
    wl = m.name2id(sim.OBJ_JOINT, "wl")
    assert m.dof_M0[m.jnt_dofadr[wl]] == pytest.approx(0.4 * 0.5 * 0.1 ** 2, rel=1e-9)
    # velocity actuators: gain kv, bias -kv qvel
    np.testing.assert_allclose(m.actuator_gainprm[:, 0], 5)
    np.testing.assert_allclose(m.actuator_biasprm[:, 2], -5)


@pytest.mark.parametrize("scene, expected", [
    # C3: 7 arm capsules (contype 2 / conaffinity 1) x floor + 4 env boxes (class env: 1 / 2); arm-arm
    # 2 & 1 = 0 both ways; env geoms share the world body; the pedestal has contype 0
    ("arm7_lidar", 7 * 5),
    # C5: floor (1/1) x arm 7 + floor x boxes 8 + arm x boxes 7 * 8 (2 & 3) + box x box C(8,2)
    ("arm_boxes", 7 + 8 + 56 + 28),
    # C4: caster and two wheels (1/1) x 8 world geoms (floor, 4 walls, 2 pillars, post); caster-wheel
    # pairs are parent-child bodies (filterparent); wheel-wheel collide; the chassis has contype 0
    ("mobile_base", 3 * 8 + 1),
])
def test_candidate_collision_pairs(scene, expected):
    m = sim.Model.load(SCENES / f"{scene}.xml")
    pairs = np.stack([m.pair_geom1, m.pair_geom2], axis=1)
    assert m.npair == expected
    np.testing.assert_array_equal(pairs, binding.candidate_pairs(m))
    # lower geom type first (the narrow phase's convention)
    assert np.all(m.geom_type[pairs[:, 0]] <= m.geom_type[pairs[:, 1]])
    # no pair within one body, no parent-child pair below the world
    for g1, g2 in pairs:
        b1, b2 = m.geom_bodyid[g1], m.geom_bodyid[g2]
        assert b1 != b2
        if b1 and b2:
            assert m.body_parentid[b1] != b2 and m.body_parentid[b2] != b1


def test_candidate_pairs_follow_filter_flags():
    """<flag filterparent="disable"/> admits parent-child pairs; <flag contact="disable"/> removes all"""
    base = (SCENES / "mobile_base.xml").read_text()
    m = sim.Model.from_string(base.replace('<option timestep="0.002"', '<option><flag filterparent="disable"/></option>'
                                           '<option timestep="0.002"', 1), str(SCENES))
    assert m.npair == 3 * 8 + 1 + 2          # + caster-wheel_l, caster-wheel_r
    np.testing.assert_array_equal(np.stack([m.pair_geom1, m.pair_geom2], 1), binding.candidate_pairs(m))
    m = sim.Model.from_string(base.replace('<option timestep="0.002"', '<option><flag contact="disable"/></option>'
                                           '<option timestep="0.002"', 1), str(SCENES))
    assert m.npair == 0 and len(binding.candidate_pairs(m)) == 0
