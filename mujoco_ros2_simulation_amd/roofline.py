"""Algorithmic work per env-step, for roofline reporting (DESIGN.md §4 states these numbers).

Counts are *useful* floating-point operations of the restated algorithm (oracle/oracle.c), an FMA
counted as 2, sqrt/div as 1, derived from the model's structure — not instruction counts of the
kernel (bounding-sphere pre-tests, index math and shuffles are overhead, not work).  Bytes are the
algorithmic HBM traffic of one fused launch (state read once, written once, sensordata written every
step) divided by its steps.
"""
from __future__ import annotations

from . import sim

# per-item flop counts of the restated primitives
RAY_SETUP = 90          # site world pose: quat mul (28) + rotate (30) + quat->mat z column (~30)
RAY_LOCAL = 33          # world ray -> geom frame: 3 sub + 2 transposed 3x3 mat-vec
RAY_PRIM = {sim.GEOM_PLANE: 12, sim.GEOM_SPHERE: 22, sim.GEOM_BOX: 48, sim.GEOM_CAPSULE: 70,
            sim.GEOM_CYLINDER: 50, sim.GEOM_ELLIPSOID: 34}
FK_BODY = 150           # parent compose (rotate 30 + quat mul 28 + add 3) + quat->mat (30) + ipos, inertia rot (~60)
FK_JOINT = 90           # anchor/axis (60) + axis-angle quat, compose (~30)
GEOM_POSE = 88          # rotate + quat mul + quat->mat
CINERT = 40             # parallel-axis terms
CRB_PAIR = 48           # 6x10 inertia-vector product (36) + 6-dot (12)
COMVEL_DOF = 42         # crossMotion (30) + axpy (12)
RNE_BODY = 140          # 2 inertia-vec (72) + crossForce (30) + accumulate (~38)
ACT = 12
PGS_ROW = 4             # per dof per row update: dot (2) + axpy (2)
COLLIDE_PAIR = 10       # bounding-sphere test per candidate pair


def flops_per_env_step(m: "sim.Model", nefc: int = None, pgs_iters: float = None) -> float:
    nv = m.nv
    f = 0.0
    # kinematics, com quantities, mass matrix and its factor/solves
    f += (m.nbody - 1) * (FK_BODY + CINERT) + m.njnt * FK_JOINT + m.ngeom * GEOM_POSE
    nmpair = sum(1 for i in range(nv) for _ in _ancestors(m, i))
    f += nmpair * CRB_PAIR + (m.nbody - 1) * 10 * 2
    f += nv ** 3 / 3 * 2 + 2 * (2 * nv * nv)          # Cholesky + two triangular solve pairs
    f += nv * COMVEL_DOF + (m.nbody - 1) * RNE_BODY + nv * 12
    f += m.nu * ACT + nv * 8                           # actuation, passive, qfrc_smooth
    # constraints: friction loss + limits present every step, contacts when active
    if nefc is None:
        nefc = int((m.dof_frictionloss > 0).sum())
    f += nefc * (2 * nv * nv + 6 * nv + 40)            # row build, M^-1 J', ARii, aref, b
    iters = pgs_iters if pgs_iters is not None else (2 if nefc else 0)
    f += iters * nefc * (PGS_ROW * nv + 10)
    # integrator (implicitfast / Euler with damping): refactor + solve + advance
    f += nv ** 3 / 3 * 2 + 2 * nv * nv + 6 * nv
    # collision broad phase is a handful of candidate pairs; narrow phase only when close
    # sensors: rangefinders dominate
    rf = [i for i in range(m.nsensor) if m.sensor_type[i] == sim.SENS_RANGEFINDER]
    per_ray = RAY_SETUP
    for g in range(m.ngeom):
        if m.geom_rgba[g, 3] == 0:
            continue
        per_ray += RAY_LOCAL + RAY_PRIM.get(int(m.geom_type[g]), 40)
    # a ray skips the geoms of its own body
    f += len(rf) * per_ray
    return f


def bytes_per_env_step(m: "sim.Model", steps_per_launch: int) -> float:
    state_in = 4 * (m.nq + m.nv + m.nu + m.nv + m.nv) + 8      # qpos qvel ctrl qfrc_applied warmstart time
    state_out = 4 * (m.nq + m.nv + m.nv + m.nv + m.nv) + 8 + 4 + 48 * m.ngeom
    sens = 4 * m.nsensordata
    return (state_in + state_out) / steps_per_launch + sens


def _ancestors(m, i):
    j = i
    while j >= 0:
        yield j
        j = m.dof_parentid[j]


# SURVEY.md §8(d) per-unit algorithmic figures (flops, bytes per env-step) for the configs; the
# bench's roofline uses these, the structural count above is reported beside them for reference
SURVEY_PER_ENV_STEP = {
    "scene": (2.0e3, 72.0),          # C2: reference 2-DoF scene, dynamics only
    "arm7_lidar": (1.9e5, 1692.0),   # C3: 7-DoF arm + 360-ray lidar
    # C3 with a 1080-beam lidar: SURVEY's C3 formula (rays x 12 geoms x ~40 + ~15k dynamics) at 1080
    # rays; bytes: state 7 x 9 floats + 1080 ranges
    "arm7_lidar1080": (1080 * 12 * 40 + 1.5e4, 4.0 * (63 + 1080 + 3)),
    "arm_boxes": (3.3e6, 1852.0),    # C5: arm + 8 free boxes, PGS 50 iterations
}

PEAK_FP32_TFLOPS = 157.3   # MI355X fp32 vector (= fp32 MFMA) peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0      # HBM3E spec peak
