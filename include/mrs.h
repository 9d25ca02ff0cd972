/*
 * mrs.h — C ABI of the MI355X batched rigid-body simulator (library libmrs.so).
 *
 * This is the boundary the re-implemented `mujoco_ros2_control/MujocoSystemInterface` plugin calls
 * instead of MuJoCo.  Every entry point names the reference call site it replaces (paths relative
 * to the reference repository).  Conventions: opaque handles, int status codes
 * (MRS_OK = 0, negative = error, message via mrs_last_error()), no exceptions across the ABI,
 * caller-owned host buffers in fp64 (mjtNum), one batch handle used by one thread at a time (the
 * plugin serialises with its own mutex, as the reference serialises with sim_mutex_).
 * Environment e of a batch is an independent mjData; the plugin maps ROS-visible state to env 0.
 * Device state is fp32, structure-of-arrays per field, env-major inside a field
 * (qpos[e * nq + i]); host get/set convert.
 */
#ifndef MRS_H
#define MRS_H

#include "mrs_model.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mrs_model mrs_model; /* compiled model (mjModel analogue) */
typedef struct mrs_batch mrs_batch; /* N environments resident on one GPU (N x mjData analogue) */

enum {
  MRS_OK = 0,
  MRS_ERR_INVALID = -1,     /* bad argument / handle / range */
  MRS_ERR_LOAD = -2,        /* model could not be parsed or compiled */
  MRS_ERR_DEVICE = -3,      /* HIP runtime error or no usable GPU */
  MRS_ERR_UNSUPPORTED = -4  /* feature outside the implemented subset */
};

/* batch state fields addressable through mrs_batch_device_ptr / get / set */
enum {
  MRS_FIELD_QPOS = 0,          /* nq,  fp32 */
  MRS_FIELD_QVEL = 1,          /* nv,  fp32 */
  MRS_FIELD_CTRL = 2,          /* nu,  fp32 */
  MRS_FIELD_QFRC_APPLIED = 3,  /* nv,  fp32 */
  MRS_FIELD_QACC_WARMSTART = 4,/* nv,  fp32 */
  MRS_FIELD_QACC = 5,          /* nv,  fp32 (output) */
  MRS_FIELD_QFRC_ACTUATOR = 6, /* nv,  fp32 (output) */
  MRS_FIELD_SENSORDATA = 7,    /* nsensordata, fp32 (output) */
  MRS_FIELD_TIME = 8,          /* 1,   fp64 */
  MRS_FIELD_WARNING = 9,       /* 4,   int32: counts of bad qpos, bad qvel, bad qacc (auto-resets), and of
                                  helper-wave signal timeouts (an internal protocol fault: the step then
                                  built its rows inline; 0 in every correct run) */
  MRS_FIELD_NCON = 10,         /* 1,   int32: contacts found in the last step (output) */
  MRS_FIELD_SOLVER_NITER = 11, /* 1,   int32: constraint solver iterations of the last step (mjData.solver_niter) */
  MRS_FIELD_COUNT = 12
};

/* last error message of the calling thread ("" if none) */
const char* mrs_last_error(void);
/* status code (MRS_OK or MRS_ERR_*) of the calling thread's last call, for the entry points that
 * return a handle (NULL on failure) rather than a code */
int mrs_last_status(void);

/* ------------------------------------------------------------------ model
 * replaces mj_loadXML (src/mujoco_system_interface.cpp:318).  The reference's other branch, a path
 * ending in ".mjb" loaded by mj_loadModel (:307-310), is not supported: such a path fails with
 * MRS_ERR_UNSUPPORTED (mrs_last_status) and "could not load binary model ..." in `error` */
mrs_model* mrs_model_load_xml(const char* path, char* error, int error_len);
/* replaces mj_parseXMLString + mj_compile (src/mujoco_system_interface.cpp:398-399, model from the
 * /mujoco_robot_description topic); `basedir` resolves <include> (may be NULL) */
mrs_model* mrs_model_load_xml_string(const char* xml, const char* basedir, char* error,
                                     int error_len);
/* replaces mj_deleteModel (src/mujoco_system_interface.cpp:512) */
void mrs_model_free(mrs_model* m);
/* deep copy of a compiled model (mj_copyModel behind get_model, src/mujoco_system_interface.cpp:
 * 1794-1798); NULL on a null argument */
mrs_model* mrs_model_copy(const mrs_model* m);
/* read-only view of the compiled arrays (mjModel field access throughout the plugin, e.g.
 * jnt_qposadr at src/mujoco_system_interface.cpp:1224); valid while `m` lives */
int mrs_model_view_get(const mrs_model* m, mrs_model_view* out);
/* opt into this restatement's own solver variants (MRS_RESTATE_* bits of mrs_model.h; 0, the
 * default, follows the upstream rules); batches created afterwards use them */
int mrs_model_set_restate(mrs_model* m, int flags);
/* replaces mj_name2id (src/mujoco_system_interface.cpp:1193,1213,1496-1497,1527-1529);
 * objtype is MRS_OBJ_*; returns -1 if not found */
int mrs_name2id(const mrs_model* m, int objtype, const char* name);
/* replaces mj_id2name (src/mujoco_lidar.cpp:139); NULL if unnamed or out of range */
const char* mrs_id2name(const mrs_model* m, int objtype, int id);
/* replaces getActuatorType (src/mujoco_system_interface.cpp:433-460):
 * 1 MOTOR, 2 POSITION, 3 VELOCITY, 4 CUSTOM, 0 UNKNOWN (same numbering as ActuatorType) */
int mrs_actuator_type(const mrs_model* m, int actuator_id);

/* ------------------------------------------------------------------ batch
 * replaces mj_makeData (src/mujoco_system_interface.cpp:686-687) for n_envs environments on HIP
 * device `device`; all envs start at qpos0 (mj_resetData) */
mrs_batch* mrs_batch_create(const mrs_model* m, int n_envs, int device);
/* replaces mj_deleteData (src/mujoco_system_interface.cpp:504-509) */
void mrs_batch_free(mrs_batch* b);
int mrs_batch_num_envs(const mrs_batch* b);
/* use an external HIP stream (hipStream_t) for all batch work; NULL = the batch's own stream */
int mrs_batch_set_stream(mrs_batch* b, void* hip_stream);
/* mj_resetData / mj_resetDataKeyframe for envs [env0, env0+n): key < 0 resets to qpos0 */
int mrs_batch_reset(mrs_batch* b, int key, int env0, int n);

/* host <-> device state copies for envs [env0, env0+n), host layout [n][dim] fp64.
 * set_* replace the control->sim copies mju_copy(ctrl/qfrc_applied) at
 * src/mujoco_system_interface.cpp:1688-1689,1728-1729 and set_initial_pose/keyframe writes
 * (:1611-1614,1617-1626); get_* replace the reads of mj_data_control_ in read()
 * (:1057-1098) and of sensordata in MujocoLidar::update (src/mujoco_lidar.cpp:247-250). */
int mrs_batch_set_field(mrs_batch* b, int field, const double* host, int env0, int n);
int mrs_batch_get_field(mrs_batch* b, int field, double* host, int env0, int n);
/* device pointer of a field (for zero-copy use from torch / RCCL); layout [n_envs][dim] */
void* mrs_batch_device_ptr(mrs_batch* b, int field);
/* copy ctrl for all envs from a device buffer [n_envs][nu] fp32 (device-resident actions) */
int mrs_batch_set_ctrl_device(mrs_batch* b, const float* d_ctrl);
/* zero-copy form of the same write (a policy's output tensor as the sim's ctrl): the following step
 * and forward launches read ctrl from the caller's device buffer [n_envs][nu] fp32, stream-ordered
 * on the batch stream, until another buffer is bound, NULL is bound, or ctrl is set by
 * mrs_batch_set_field / mrs_batch_set_ctrl_device (which return to the batch's own buffer).  Reads
 * of the ctrl field return the bound buffer's values.  The buffer must stay valid while bound. */
int mrs_batch_bind_ctrl_device(mrs_batch* b, const float* d_ctrl);

/* replaces mj_step (src/mujoco_system_interface.cpp:1691,1731): advance every env n_steps times,
 * fused in one launch; ctrl / qfrc_applied are held constant (zero-order hold) across the n steps,
 * exactly as PhysicsLoop holds them between write() calls.  Asynchronous on the batch stream. */
int mrs_batch_step(mrs_batch* b, int n_steps);
/* replaces mj_forward (src/mujoco_system_interface.cpp:741,1771): recompute outputs (sensordata,
 * qfrc_actuator, qacc) for the current state without integrating */
int mrs_batch_forward(mrs_batch* b);
/* depth image of camera `cam` for envs [env0, env0+n): host out [n][H][W] fp32, rows already
 * flipped to ROS order and linearised to eye-space z (replaces mjr_render + mjr_readPixels +
 * the linearisation loop of src/mujoco_cameras.cpp:211-240) */
int mrs_batch_render_depth(mrs_batch* b, int cam, int env0, int n, float* host_out);
/* same, into a device buffer [n][H][W] (stays in HBM) */
int mrs_batch_render_depth_device(mrs_batch* b, int cam, int env0, int n, float* d_out);
/* depth and colour in one pass (the RGB8 image of src/mujoco_cameras.cpp:211-240): depth as above,
 * rgb [n][H][W][3] uint8, ROS row order, each pixel's nearest geom shaded by MuJoCo's fixed-function
 * lighting model restated per pixel (headlight and model lights, shadows, materials, builtin
 * textures; the skybox where nothing is hit) -- not an OpenGL raster match */
int mrs_batch_render_rgbd(mrs_batch* b, int cam, int env0, int n, float* host_depth, unsigned char* host_rgb);
/* same, into device buffers */
int mrs_batch_render_rgbd_device(mrs_batch* b, int cam, int env0, int n, float* d_depth, unsigned char* d_rgb);
/* camera pipeline (the reference's rendering thread: mjv_copyData of the live data under the sim
 * mutex, then mjv_updateScene + mjr_render of the copy while PhysicsLoop steps on,
 * src/mujoco_cameras.cpp:204-215): snapshot the poses of the last step on the batch stream, then
 * render depth (and colour when d_rgb is not NULL) from the snapshot on the batch's own render stream,
 * concurrently with the steps queued after this call.  Device buffers as mrs_batch_render_rgbd_device.
 * A later snapshot waits until the previous asynchronous render has read the old one. */
int mrs_batch_render_async(mrs_batch* b, int cam, int env0, int n, float* d_depth, unsigned char* d_rgb);
/* order the batch stream after the last asynchronous render (its frames are complete for any work
 * queued on the batch stream afterwards; mrs_batch_sync also waits for it) */
int mrs_batch_render_wait(mrs_batch* b);
/* mjData.contact of env `env` after its last step / forward (the output of mj_collision, SURVEY.md
 * §8a row a2.3): up to `max` contacts in mj_collision's order -- geom [max][2] int32 (geom1, geom2,
 * the lower geom type first), dist [max], pos [max][3], frame [max][9] fp64 (normal = frame[0:3]);
 * any output pointer may be NULL.  Returns ncon (which may exceed `max`) or a negative error code. */
int mrs_batch_get_contacts(mrs_batch* b, int env, int max, int* geom, double* dist, double* pos,
                           double* frame);
/* mjData.efc_* of env `env` after its last step / forward (the rows mj_makeConstraint built and the
 * solver's forces): up to `max` rows in mj_makeConstraint's order --
 * type [max] int32 (1 friction loss, 2 joint limit, 3 contact), J [max][nv], R [max], aref [max],
 * force [max] fp64; any output pointer may be NULL.  Returns nefc (which may exceed `max`), or
 * MRS_ERR_UNSUPPORTED for the layouts that keep no dense rows (the register friction-loss path of
 * models without contacts or active limits, and PGS in blocked mode, whose rows are sparse). */
int mrs_batch_get_efc(mrs_batch* b, int env, int max, int* type, double* J, double* R, double* aref,
                      double* force);
/* fp32 state field rows of envs [env0, env0+n) into a device buffer [n][dim], asynchronous on the
 * batch stream (observations for the end-of-step gather stay in HBM; no reference counterpart: the
 * reference copies mjData on the host, src/mujoco_system_interface.cpp:1759) */
int mrs_batch_get_field_device(mrs_batch* b, int field, float* d_out, int env0, int n);
/* wait for all queued batch work */
int mrs_batch_sync(mrs_batch* b);
/* duration in ms of the last step / render kernel measured with HIP events on the batch stream
 * (kind 0 = step, 1 = depth), -1 if unavailable (no such launch yet, or its kind is not timed) */
double mrs_batch_last_kernel_ms(mrs_batch* b, int kind);
/* which launches the batch brackets with its own HIP events for mrs_batch_last_kernel_ms: bit 0 step
 * launches, bit 1 frames (default 2: frames only).  A timed step launch costs ~10 us (a C3 10-step
 * launch 0.420 vs 0.410 ms), so step launches are timed only when asked for */
int mrs_batch_set_timing(mrs_batch* b, int mask);
/* diagnostics (no reference counterpart): per-phase wave-cycle totals of the step kernel since the
 * last reset, in phase order kinematics, com_pos, make_M, cholesky, com_vel, rne, smooth_forces,
 * collision, constraints, sensors, integrate, checks.  Only a library built with
 * -DMRS_PHASE_TIMING records them; returns the number of phases written (0 otherwise, <0 on error). */
int mrs_debug_phase_cycles(double* out, int n, int reset);
/* diagnostics: the batch's kernel configuration -- out[0] lanes per env (group width), [1] LDS floats
 * per env, [2] scratch floats per env, [3] blocked mode (tree-blocked M + sparse constraint rows),
 * [4] dof slots per constraint row (pipe width), [5] constraint-row capacity, [6] contact capacity,
 * [7] kinematic trees with dofs, [8] workgroup-shared LDS floats, [9] lidar rays read from the
 * workgroup's LDS table (1) or the model block (0), [10] one workgroup per CU (16-lane groups kept for
 * tables past the two-per-CU budget), [11] waves per workgroup of a 16-lane batch (0 otherwise),
 * [12] helper waves (collision, rows, rays and the integrator factor beside the dynamics).  Returns
 * the number of values written. */
int mrs_debug_batch_layout(const mrs_batch* b, int* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* MRS_H */
