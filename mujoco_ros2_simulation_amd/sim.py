"""ctypes binding of the C ABI (include/mrs.h) — the host-side mirror used by tests, bench and the
plugin harness.  The product path is libmrs.so (HIP kernels for gfx950); there is no CPU fallback:
if the library or a GPU is missing, the calls raise.

Reference mapping (reference repo paths):
  Model.load        -> mj_loadXML            src/mujoco_system_interface.cpp:318
  Model.from_string -> mj_parseXMLString+mj_compile  :398-399
  Model.name2id     -> mj_name2id            :1193,1213,1496-1497,1527-1529
  Batch             -> N x mjData             mj_makeData :686-687
  Batch.step        -> mj_step               :1691,1731
  Batch.forward     -> mj_forward            :741,1771
  Batch.render_depth-> mjr_render+mjr_readPixels+linearise  src/mujoco_cameras.cpp:211-240
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["MRS_LIB"]) if os.environ.get("MRS_LIB") else _PKG / "libmrs.so"

# enums mirrored from include/mrs_model.h / include/mrs.h
GEOM_PLANE, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE, GEOM_ELLIPSOID, GEOM_CYLINDER, GEOM_BOX, GEOM_MESH = range(8)
JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = range(4)
OBJ_BODY, OBJ_JOINT, OBJ_GEOM, OBJ_SITE, OBJ_CAMERA, OBJ_ACTUATOR, OBJ_SENSOR = 1, 3, 5, 6, 7, 19, 20
OBJ_TENDON = 18
SENS_ACCELEROMETER, SENS_GYRO, SENS_FORCE, SENS_TORQUE, SENS_RANGEFINDER = 1, 3, 4, 5, 7
SENS_JOINTPOS, SENS_JOINTVEL, SENS_ACTUATORFRC, SENS_FRAMEPOS, SENS_FRAMEQUAT = 9, 10, 15, 25, 26
BIAS_NONE, BIAS_AFFINE = 0, 1
RESTATE_NEWTON_REFINE, RESTATE_PGS_ELLIPTIC_BLOCK, RESTATE_NO_MPR_POLISH, RESTATE_NO_MULTICCD = 1, 2, 4, 8
(FIELD_QPOS, FIELD_QVEL, FIELD_CTRL, FIELD_QFRC_APPLIED, FIELD_QACC_WARMSTART, FIELD_QACC,
 FIELD_QFRC_ACTUATOR, FIELD_SENSORDATA, FIELD_TIME, FIELD_WARNING, FIELD_NCON, FIELD_SOLVER_NITER) = range(12)
# ActuatorType (include/mujoco_ros2_control/data.hpp:43-51 numbering)
ACT_UNKNOWN, ACT_MOTOR, ACT_POSITION, ACT_VELOCITY, ACT_CUSTOM = range(5)

MRS_OK = 0
ERRORS = {-1: "invalid argument", -2: "load error", -3: "device error", -4: "unsupported"}


class MrsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


# (name, kind, size-expression) in exactly the order of struct mrs_model_view
_SIZES = ["nq", "nv", "nu", "na", "nbody", "njnt", "ngeom", "nsite", "ncam", "nsensor", "nsensordata", "nkey",
          "nM", "max_depth", "npair"]
_ARRAYS = [
    ("body_parentid", "i", "nbody", 1), ("body_rootid", "i", "nbody", 1), ("body_weldid", "i", "nbody", 1),
    ("body_jntnum", "i", "nbody", 1), ("body_jntadr", "i", "nbody", 1), ("body_dofnum", "i", "nbody", 1),
    ("body_dofadr", "i", "nbody", 1), ("body_geomnum", "i", "nbody", 1), ("body_geomadr", "i", "nbody", 1),
    ("body_depth", "i", "nbody", 1),
    ("body_pos", "d", "nbody", 3), ("body_quat", "d", "nbody", 4), ("body_ipos", "d", "nbody", 3),
    ("body_iquat", "d", "nbody", 4), ("body_mass", "d", "nbody", 1), ("body_subtreemass", "d", "nbody", 1),
    ("body_inertia", "d", "nbody", 3), ("body_invweight0", "d", "nbody", 2), ("body_gravcomp", "d", "nbody", 1),
    ("jnt_type", "i", "njnt", 1), ("jnt_qposadr", "i", "njnt", 1), ("jnt_dofadr", "i", "njnt", 1),
    ("jnt_bodyid", "i", "njnt", 1), ("jnt_limited", "i", "njnt", 1), ("jnt_actfrclimited", "i", "njnt", 1),
    ("jnt_pos", "d", "njnt", 3), ("jnt_axis", "d", "njnt", 3), ("jnt_stiffness", "d", "njnt", 1),
    ("jnt_range", "d", "njnt", 2), ("jnt_actfrcrange", "d", "njnt", 2), ("jnt_margin", "d", "njnt", 1),
    ("jnt_solref", "d", "njnt", 2), ("jnt_solimp", "d", "njnt", 5),
    ("dof_bodyid", "i", "nv", 1), ("dof_jntid", "i", "nv", 1), ("dof_parentid", "i", "nv", 1),
    ("dof_armature", "d", "nv", 1), ("dof_damping", "d", "nv", 1), ("dof_frictionloss", "d", "nv", 1),
    ("dof_solref", "d", "nv", 2), ("dof_solimp", "d", "nv", 5), ("dof_invweight0", "d", "nv", 1),
    ("dof_M0", "d", "nv", 1),
    ("geom_type", "i", "ngeom", 1), ("geom_contype", "i", "ngeom", 1), ("geom_conaffinity", "i", "ngeom", 1),
    ("geom_condim", "i", "ngeom", 1), ("geom_bodyid", "i", "ngeom", 1), ("geom_group", "i", "ngeom", 1),
    ("geom_priority", "i", "ngeom", 1),
    ("geom_size", "d", "ngeom", 3), ("geom_pos", "d", "ngeom", 3), ("geom_quat", "d", "ngeom", 4),
    ("geom_rbound", "d", "ngeom", 1), ("geom_friction", "d", "ngeom", 3), ("geom_margin", "d", "ngeom", 1),
    ("geom_gap", "d", "ngeom", 1), ("geom_solmix", "d", "ngeom", 1), ("geom_solref", "d", "ngeom", 2),
    ("geom_solimp", "d", "ngeom", 5), ("geom_rgba", "d", "ngeom", 4),
    ("site_bodyid", "i", "nsite", 1), ("site_pos", "d", "nsite", 3), ("site_quat", "d", "nsite", 4),
    ("cam_bodyid", "i", "ncam", 1), ("cam_resolution", "i", "ncam", 2), ("cam_pos", "d", "ncam", 3),
    ("cam_quat", "d", "ncam", 4), ("cam_fovy", "d", "ncam", 1),
    ("actuator_trntype", "i", "nu", 1), ("actuator_dyntype", "i", "nu", 1), ("actuator_gaintype", "i", "nu", 1),
    ("actuator_biastype", "i", "nu", 1), ("actuator_trnid", "i", "nu", 2), ("actuator_ctrllimited", "i", "nu", 1),
    ("actuator_forcelimited", "i", "nu", 1),
    ("actuator_gear", "d", "nu", 6), ("actuator_gainprm", "d", "nu", 10), ("actuator_biasprm", "d", "nu", 10),
    ("actuator_ctrlrange", "d", "nu", 2), ("actuator_forcerange", "d", "nu", 2),
    ("sensor_type", "i", "nsensor", 1), ("sensor_objtype", "i", "nsensor", 1), ("sensor_objid", "i", "nsensor", 1),
    ("sensor_dim", "i", "nsensor", 1), ("sensor_adr", "i", "nsensor", 1), ("sensor_cutoff", "d", "nsensor", 1),
    ("qpos0", "d", "nq", 1), ("qpos_spring", "d", "nq", 1),
    ("key_time", "d", "nkey", 1), ("key_qpos", "d", "nkey", "nq"), ("key_qvel", "d", "nkey", "nv"),
    ("key_ctrl", "d", "nkey", "nu"),
    ("pair_geom1", "i", "npair", 1), ("pair_geom2", "i", "npair", 1),
]
# mesh block (after the arrays above in struct mrs_model_view)
_MESH_SIZES = ["nmesh", "nmeshvert", "nmeshface", "nmeshhull"]
_MESH_ARRAYS = [
    ("geom_dataid", "i", "ngeom", 1), ("mesh_vertadr", "i", "nmesh", 1), ("mesh_vertnum", "i", "nmesh", 1),
    ("mesh_faceadr", "i", "nmesh", 1), ("mesh_facenum", "i", "nmesh", 1), ("mesh_hulladr", "i", "nmesh", 1),
    ("mesh_hullnum", "i", "nmesh", 1), ("mesh_face", "i", "nmeshface", 3), ("mesh_hull", "i", "nmeshhull", 1),
    ("mesh_vert", "d", "nmeshvert", 3),
]
# explicit contact pairs and excluded body pairs (after the mesh block)
_CONTACT_SIZES = ["nexpair", "nexclude"]
_CONTACT_ARRAYS = [
    ("expair_geom1", "i", "nexpair", 1), ("expair_geom2", "i", "nexpair", 1), ("expair_dim", "i", "nexpair", 1),
    ("exclude_body1", "i", "nexclude", 1), ("exclude_body2", "i", "nexclude", 1),
    ("expair_friction", "d", "nexpair", 5), ("expair_solref", "d", "nexpair", 2), ("expair_solimp", "d", "nexpair", 5),
    ("expair_margin", "d", "nexpair", 1), ("expair_gap", "d", "nexpair", 1),
]
# equality constraints (after the contact block)
_EQ_SIZES = ["neq"]
_EQ_ARRAYS = [
    ("eq_type", "i", "neq", 1), ("eq_obj1id", "i", "neq", 1), ("eq_obj2id", "i", "neq", 1), ("eq_active0", "i", "neq", 1),
    ("eq_solref", "d", "neq", 2), ("eq_solimp", "d", "neq", 5), ("eq_data", "d", "neq", 11),
]
EQ_CONNECT, EQ_WELD, EQ_JOINT = 0, 1, 2
# rendering (after the equality block; vis_headlight is a fixed double[10] before the sizes)
_REND_SIZES = ["nlight", "ntex", "nmat"]
_REND_ARRAYS = [
    ("light_directional", "i", "nlight", 1), ("light_castshadow", "i", "nlight", 1), ("light_active", "i", "nlight", 1),
    ("tex_type", "i", "ntex", 1), ("tex_builtin", "i", "ntex", 1), ("tex_mark", "i", "ntex", 1),
    ("tex_width", "i", "ntex", 1), ("tex_height", "i", "ntex", 1), ("mat_texid", "i", "nmat", 1),
    ("mat_texuniform", "i", "nmat", 1), ("geom_matid", "i", "ngeom", 1),
    ("light_pos", "d", "nlight", 3), ("light_dir", "d", "nlight", 3), ("light_ambient", "d", "nlight", 3),
    ("light_diffuse", "d", "nlight", 3), ("light_specular", "d", "nlight", 3), ("light_attenuation", "d", "nlight", 3),
    ("light_cutoff", "d", "nlight", 1), ("light_exponent", "d", "nlight", 1), ("tex_rgb1", "d", "ntex", 3),
    ("tex_rgb2", "d", "ntex", 3), ("tex_markrgb", "d", "ntex", 3), ("mat_rgba", "d", "nmat", 4),
    ("mat_texrepeat", "d", "nmat", 2), ("mat_specular", "d", "nmat", 1), ("mat_shininess", "d", "nmat", 1),
    ("mat_emission", "d", "nmat", 1),
]
TEX_2D, TEX_CUBE, TEX_SKYBOX = 0, 1, 2
# fixed tendons (after the rendering block)
_TEN_SIZES = ["ntendon", "nwrap"]
_TEN_ARRAYS = [
    ("tendon_adr", "i", "ntendon", 1), ("tendon_num", "i", "ntendon", 1), ("tendon_limited", "i", "ntendon", 1),
    ("wrap_objid", "i", "nwrap", 1), ("wrap_prm", "d", "nwrap", 1), ("tendon_range", "d", "ntendon", 2),
    ("tendon_margin", "d", "ntendon", 1), ("tendon_solref_lim", "d", "ntendon", 2),
    ("tendon_solimp_lim", "d", "ntendon", 5), ("tendon_frictionloss", "d", "ntendon", 1),
    ("tendon_solref_fri", "d", "ntendon", 2), ("tendon_solimp_fri", "d", "ntendon", 5),
    ("tendon_stiffness", "d", "ntendon", 1), ("tendon_damping", "d", "ntendon", 1),
    ("tendon_lengthspring", "d", "ntendon", 2), ("tendon_invweight0", "d", "ntendon", 1),
    ("tendon_length0", "d", "ntendon", 1),
]
TRN_JOINT, TRN_TENDON = 0, 3
# mesh hull polygons (after the tendon block)
_POLY_SIZES = ["nmeshpoly", "nmeshpolyvert"]
_POLY_ARRAYS = [
    ("mesh_polyadr", "i", "nmesh", 1), ("mesh_polynum", "i", "nmesh", 1), ("mesh_polyvertadr", "i", "nmeshpoly", 1),
    ("mesh_polyvertnum", "i", "nmeshpoly", 1), ("mesh_polyvert", "i", "nmeshpolyvert", 1),
    ("mesh_polynormal", "d", "nmeshpoly", 3),
]


class ModelView(C.Structure):
    _fields_ = ([(n, C.c_int) for n in _SIZES] +
                [("timestep", C.c_double), ("gravity", C.c_double * 3), ("tolerance", C.c_double),
                 ("impratio", C.c_double), ("ls_tolerance", C.c_double),
                 ("integrator", C.c_int), ("solver", C.c_int), ("iterations", C.c_int), ("disableflags", C.c_int),
                 ("cone", C.c_int), ("ls_iterations", C.c_int), ("restate", C.c_int),
                 ("stat_extent", C.c_double), ("stat_center", C.c_double * 3), ("stat_meaninertia", C.c_double),
                 ("vis_znear", C.c_double), ("vis_zfar", C.c_double)] +
                [(n, C.POINTER(C.c_int) if k == "i" else C.POINTER(C.c_double)) for n, k, _, _ in _ARRAYS] +
                [(n, C.c_int) for n in _MESH_SIZES] +
                [(n, C.POINTER(C.c_int) if k == "i" else C.POINTER(C.c_double)) for n, k, _, _ in _MESH_ARRAYS] +
                [(n, C.c_int) for n in _CONTACT_SIZES] +
                [(n, C.POINTER(C.c_int) if k == "i" else C.POINTER(C.c_double)) for n, k, _, _ in _CONTACT_ARRAYS] +
                [(n, C.c_int) for n in _EQ_SIZES] +
                [(n, C.POINTER(C.c_int) if k == "i" else C.POINTER(C.c_double)) for n, k, _, _ in _EQ_ARRAYS] +
                [("vis_headlight", C.c_double * 10)] + [(n, C.c_int) for n in _REND_SIZES] +
                [(n, C.POINTER(C.c_int) if k == "i" else C.POINTER(C.c_double)) for n, k, _, _ in _REND_ARRAYS] +
                [(n, C.c_int) for n in _TEN_SIZES] +
                [(n, C.POINTER(C.c_int) if k == "i" else C.POINTER(C.c_double)) for n, k, _, _ in _TEN_ARRAYS] +
                [(n, C.c_int) for n in _POLY_SIZES] +
                [(n, C.POINTER(C.c_int) if k == "i" else C.POINTER(C.c_double)) for n, k, _, _ in _POLY_ARRAYS])


_lib = None


def lib() -> C.CDLL:
    """Load libmrs.so (built in-tree by build.py); raises if it is missing."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise MrsError(-3, f"{LIB_PATH} not built; run `python -m mujoco_ros2_simulation_amd.build`")
        L = C.CDLL(str(LIB_PATH))
        L.mrs_last_error.restype = C.c_char_p
        L.mrs_last_status.restype = C.c_int
        L.mrs_model_load_xml.restype = C.c_void_p
        L.mrs_model_load_xml.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
        L.mrs_model_load_xml_string.restype = C.c_void_p
        L.mrs_model_load_xml_string.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        L.mrs_model_free.argtypes = [C.c_void_p]
        L.mrs_model_view_get.argtypes = [C.c_void_p, C.POINTER(ModelView)]
        L.mrs_model_set_restate.argtypes = [C.c_void_p, C.c_int]
        L.mrs_name2id.argtypes = [C.c_void_p, C.c_int, C.c_char_p]
        L.mrs_id2name.restype = C.c_char_p
        L.mrs_id2name.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.mrs_actuator_type.argtypes = [C.c_void_p, C.c_int]
        L.mrs_batch_create.restype = C.c_void_p
        L.mrs_batch_create.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.mrs_batch_free.argtypes = [C.c_void_p]
        L.mrs_batch_num_envs.argtypes = [C.c_void_p]
        L.mrs_batch_set_stream.argtypes = [C.c_void_p, C.c_void_p]
        L.mrs_batch_reset.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
        L.mrs_batch_set_field.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.mrs_batch_get_field.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.mrs_batch_device_ptr.restype = C.c_void_p
        L.mrs_batch_device_ptr.argtypes = [C.c_void_p, C.c_int]
        L.mrs_batch_set_ctrl_device.argtypes = [C.c_void_p, C.c_void_p]
        L.mrs_batch_bind_ctrl_device.argtypes = [C.c_void_p, C.c_void_p]
        L.mrs_batch_set_timing.argtypes = [C.c_void_p, C.c_int]
        L.mrs_batch_step.argtypes = [C.c_void_p, C.c_int]
        L.mrs_batch_forward.argtypes = [C.c_void_p]
        L.mrs_batch_render_depth.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.mrs_batch_render_depth_device.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.mrs_batch_render_rgbd.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.mrs_batch_render_rgbd_device.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.mrs_batch_render_async.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        L.mrs_batch_render_wait.argtypes = [C.c_void_p]
        L.mrs_batch_sync.argtypes = [C.c_void_p]
        L.mrs_batch_get_contacts.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                             C.c_void_p]
        L.mrs_batch_get_efc.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p]
        L.mrs_batch_get_field_device.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.mrs_batch_last_kernel_ms.restype = C.c_double
        L.mrs_batch_last_kernel_ms.argtypes = [C.c_void_p, C.c_int]
        L.mrs_debug_phase_cycles.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.mrs_debug_batch_layout.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        _lib = L
    return _lib


PHASES = ["kinematics", "com_pos", "make_M", "cholesky", "com_vel", "rne", "smooth_forces", "collision",
          "constraints", "sensors", "integrate", "checks", "sensors.level1", "sensors.setup", "sensors.geoms",
          "constraints.rows", "constraints.records", "constraints.warmstart", "constraints.pgs",
          "collision.narrow", "collision.out", "constraints.delassus", "records.jac", "records.solve",
          "records.rows"]


def phase_cycles(reset: bool = False) -> dict | None:
    """per-phase wave-cycle totals of the step kernel (profiling builds, -DMRS_PHASE_TIMING)"""
    out = np.zeros(len(PHASES))
    n = lib().mrs_debug_phase_cycles(out.ctypes.data_as(C.c_void_p), len(PHASES), int(reset))
    if n <= 0:
        return None
    return dict(zip(PHASES, out[:n].tolist()))


def _check(rc: int) -> None:
    if rc != MRS_OK:
        raise MrsError(rc, lib().mrs_last_error().decode())


class Model:
    """Compiled MJCF model (mjModel analogue).  Arrays are exposed as read-only numpy views."""

    def __init__(self, handle: int):
        self._h = handle
        self.view = ModelView()
        _check(lib().mrs_model_view_get(self._h, C.byref(self.view)))
        v = self.view
        for n in _SIZES + _MESH_SIZES + _CONTACT_SIZES + _EQ_SIZES + _REND_SIZES + _TEN_SIZES + _POLY_SIZES:
            setattr(self, n, getattr(v, n))
        for n in ["timestep", "tolerance", "impratio", "ls_tolerance", "ls_iterations", "restate", "integrator", "solver",
                  "iterations", "disableflags",
                  "stat_extent", "stat_meaninertia", "vis_znear", "vis_zfar"]:
            setattr(self, n, getattr(v, n))
        self.gravity = np.array(v.gravity[:])
        self.vis_headlight = np.array(v.vis_headlight[:])
        for name, kind, count, width in (_ARRAYS + _MESH_ARRAYS + _CONTACT_ARRAYS + _EQ_ARRAYS + _REND_ARRAYS +
                                         _TEN_ARRAYS + _POLY_ARRAYS):
            n = getattr(v, count)
            w = getattr(v, width) if isinstance(width, str) else width
            ptr = getattr(v, name)
            size = n * w
            if size == 0 or not ptr:
                arr = np.zeros((n, w) if (w > 1 or isinstance(width, str)) else (n,),
                               dtype=np.int32 if kind == "i" else np.float64)
            else:
                arr = np.ctypeslib.as_array(ptr, shape=(size,)).copy()
                if w > 1 or isinstance(width, str):
                    arr = arr.reshape(n, w)
            setattr(self, name, arr)

    @classmethod
    def load(cls, path: str | os.PathLike) -> "Model":
        err = C.create_string_buffer(1024)
        h = lib().mrs_model_load_xml(str(path).encode(), err, 1024)
        if not h:
            raise MrsError(lib().mrs_last_status() or -2, err.value.decode())
        return cls(h)

    @classmethod
    def from_string(cls, xml: str, basedir: str | None = None) -> "Model":
        err = C.create_string_buffer(1024)
        h = lib().mrs_model_load_xml_string(xml.encode(), (basedir or ".").encode(), err, 1024)
        if not h:
            raise MrsError(lib().mrs_last_status() or -2, err.value.decode())
        return cls(h)

    def set_restate(self, flags: int) -> None:
        """opt into this restatement's own solver variants (RESTATE_* bits; 0 = upstream rules);
        batches and oracle data created afterwards use them"""
        _check(lib().mrs_model_set_restate(self._h, int(flags)))
        _check(lib().mrs_model_view_get(self._h, C.byref(self.view)))
        self.restate = self.view.restate

    def name2id(self, objtype: int, name: str) -> int:
        return lib().mrs_name2id(self._h, objtype, name.encode())

    def id2name(self, objtype: int, i: int) -> str | None:
        r = lib().mrs_id2name(self._h, objtype, i)
        return r.decode() if r else None

    def actuator_type(self, i: int) -> int:
        return lib().mrs_actuator_type(self._h, i)

    @property
    def handle(self) -> int:
        return self._h

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.mrs_model_free(self._h)
            self._h = None


_FIELD_DIM = {
    FIELD_QPOS: "nq", FIELD_QVEL: "nv", FIELD_CTRL: "nu", FIELD_QFRC_APPLIED: "nv", FIELD_QACC_WARMSTART: "nv",
    FIELD_QACC: "nv", FIELD_QFRC_ACTUATOR: "nv", FIELD_SENSORDATA: "nsensordata", FIELD_TIME: 1, FIELD_WARNING: 4,
    FIELD_NCON: 1, FIELD_SOLVER_NITER: 1,
}


class Batch:
    """N independent environments of one model on one GPU (N x mjData analogue)."""

    def __init__(self, model: Model, n_envs: int, device: int = 0):
        self.model = model
        self.n = n_envs
        h = lib().mrs_batch_create(model.handle, n_envs, device)
        if not h:
            raise MrsError(lib().mrs_last_status() or -3, lib().mrs_last_error().decode())
        self._h = h

    def _dim(self, field: int) -> int:
        d = _FIELD_DIM[field]
        return getattr(self.model, d) if isinstance(d, str) else d

    def get(self, field: int, env0: int = 0, n: int | None = None) -> np.ndarray:
        n = self.n - env0 if n is None else n
        out = np.empty((n, self._dim(field)), dtype=np.float64)
        _check(lib().mrs_batch_get_field(self._h, field, out.ctypes.data, env0, n))
        return out

    def set(self, field: int, values, env0: int = 0) -> None:
        if self._dim(field) == 0:  # e.g. ctrl of a model without actuators
            return
        a = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, self._dim(field))
        _check(lib().mrs_batch_set_field(self._h, field, a.ctypes.data, env0, a.shape[0]))

    def reset(self, key: int = -1, env0: int = 0, n: int | None = None) -> None:
        _check(lib().mrs_batch_reset(self._h, key, env0, self.n - env0 if n is None else n))

    def layout(self) -> dict:
        """kernel configuration of this batch (diagnostics): group width, LDS and scratch floats per
        env, blocked mode, pipe width, row and contact capacity, kinematic trees"""
        out = np.zeros(14, dtype=np.int32)
        k = lib().mrs_debug_batch_layout(self._h, out.ctypes.data, 14)
        keys = ["group", "lds_floats", "scratch_floats", "blocked", "pipe_w", "max_efc", "max_con", "ntree",
                "shared_floats", "rf_common", "one_workgroup_per_cu", "waves_per_workgroup", "helper_waves",
                "fused_integrator_factor"]
        return dict(zip(keys[:k], out[:k].tolist()))

    def step(self, n_steps: int = 1) -> None:
        _check(lib().mrs_batch_step(self._h, n_steps))

    def forward(self) -> None:
        _check(lib().mrs_batch_forward(self._h))

    def sync(self) -> None:
        _check(lib().mrs_batch_sync(self._h))

    def device_ptr(self, field: int) -> int:
        return lib().mrs_batch_device_ptr(self._h, field)

    def set_ctrl_device(self, ptr: int) -> None:
        _check(lib().mrs_batch_set_ctrl_device(self._h, C.c_void_p(ptr)))

    def bind_ctrl_device(self, ptr: int | None) -> None:
        """zero-copy ctrl: the following launches read ctrl from this device buffer [n][nu] fp32
        (None: the batch's own buffer again; set / set_ctrl_device also return to it)"""
        _check(lib().mrs_batch_bind_ctrl_device(self._h, C.c_void_p(ptr) if ptr else None))

    def set_stream(self, stream_ptr: int | None) -> None:
        _check(lib().mrs_batch_set_stream(self._h, C.c_void_p(stream_ptr) if stream_ptr else None))

    def render_depth(self, cam: int, env0: int = 0, n: int = 1) -> np.ndarray:
        W, H = self.model.cam_resolution[cam]
        out = np.empty((n, H, W), dtype=np.float32)
        _check(lib().mrs_batch_render_depth(self._h, cam, env0, n, out.ctypes.data))
        return out

    def render_rgbd(self, cam: int, env0: int = 0, n: int = 1) -> tuple[np.ndarray, np.ndarray]:
        """(depth [n, H, W] fp32, rgb [n, H, W, 3] uint8) in one pass"""
        W, H = self.model.cam_resolution[cam]
        depth = np.empty((n, H, W), dtype=np.float32)
        rgb = np.empty((n, H, W, 3), dtype=np.uint8)
        _check(lib().mrs_batch_render_rgbd(self._h, cam, env0, n, depth.ctypes.data, rgb.ctypes.data))
        return depth, rgb

    def render_rgbd_device(self, cam: int, env0: int, n: int, depth_ptr: int, rgb_ptr: int) -> None:
        _check(lib().mrs_batch_render_rgbd_device(self._h, cam, env0, n, C.c_void_p(depth_ptr), C.c_void_p(rgb_ptr)))

    def render_depth_device(self, cam: int, env0: int, n: int, dptr: int) -> None:
        _check(lib().mrs_batch_render_depth_device(self._h, cam, env0, n, C.c_void_p(dptr)))

    def render_async(self, cam: int, env0: int, n: int, depth_ptr: int, rgb_ptr: int = 0) -> None:
        """snapshot the last step's poses, render from the snapshot concurrently with later steps"""
        _check(lib().mrs_batch_render_async(self._h, cam, env0, n, C.c_void_p(depth_ptr),
                                             C.c_void_p(rgb_ptr) if rgb_ptr else None))

    def render_wait(self) -> None:
        """order the batch stream after the last asynchronous render"""
        _check(lib().mrs_batch_render_wait(self._h))

    def contacts(self, env: int = 0, max_n: int = 256):
        """mjData.contact of `env` after the last step/forward: (geom [n, 2] int32, dist [n],
        pos [n, 3], frame [n, 9]) in mj_collision's order"""
        g = np.zeros((max_n, 2), dtype=np.int32)
        dist, pos, frame = np.zeros(max_n), np.zeros((max_n, 3)), np.zeros((max_n, 9))
        n = lib().mrs_batch_get_contacts(self._h, env, max_n, g.ctypes.data, dist.ctypes.data, pos.ctypes.data,
                                         frame.ctypes.data)
        if n < 0:
            _check(n)
        n = min(n, max_n)
        return g[:n], dist[:n], pos[:n], frame[:n]

    def efc(self, env: int = 0, max_n: int = 1024):
        """mjData.efc_* of `env` after the last step/forward: dict of type [n] (1 friction loss,
        2 limit, 3 contact), J [n, nv], R, aref, force [n]"""
        nv = self.model.nv
        t = np.zeros(max_n, dtype=np.int32)
        J = np.zeros((max_n, max(nv, 1)))
        R, a, f = np.zeros(max_n), np.zeros(max_n), np.zeros(max_n)
        n = lib().mrs_batch_get_efc(self._h, env, max_n, t.ctypes.data, J.ctypes.data, R.ctypes.data, a.ctypes.data,
                                    f.ctypes.data)
        if n < 0:
            _check(n)
        n = min(n, max_n)
        return {"type": t[:n], "J": J[:n, :nv], "R": R[:n], "aref": a[:n], "force": f[:n]}

    def get_device(self, field: int, dptr: int, env0: int = 0, n: int | None = None) -> None:
        """fp32 rows of `field` into a device buffer [n, dim], asynchronous on the batch stream"""
        n = self.n - env0 if n is None else n
        _check(lib().mrs_batch_get_field_device(self._h, field, C.c_void_p(dptr), env0, n))

    def set_timing(self, mask: int) -> None:
        """launches bracketed by the batch's own HIP events (bit 0 step, bit 1 frames; default 2)"""
        _check(lib().mrs_batch_set_timing(self._h, mask))

    def last_kernel_ms(self, kind: int = 0) -> float:
        return lib().mrs_batch_last_kernel_ms(self._h, kind)

    def close(self) -> None:
        if getattr(self, "_h", None) and _lib is not None:
            _lib.mrs_batch_free(self._h)
            self._h = None

    def __del__(self):
        self.close()
