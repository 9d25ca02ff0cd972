// Device-side model and per-env memory layout for the fused step kernel.
//
// The compiled fp64 model (mrs::Model) is packed on the host into one fp32 device block plus one
// int32 block; DevModel carries the counts and the device pointers (passed by value as a kernel
// argument, so counts live in SGPRs and wave-uniform array reads become scalar loads).  Host-side
// precomputation turns tree walks into flat lists: bodies grouped by depth (tree-level parallel
// passes), DFS subtree ranges (subtree sums without serial accumulation), the (dof, ancestor-dof)
// pairs of the mass matrix, the statically admissible collision pairs, friction-loss dofs,
// limited joints and rangefinder sensors.
#pragma once

#include <cstdint>

#include "../../../include/mrs_model.h"

namespace mrs {

struct DevModel {
  // sizes
  int nq, nv, nu, nbody, njnt, ngeom, nsite, ncam, nsensor, nsensordata, max_depth;
  int nfric, nlim, npair, nrf, nMpair, max_con, max_efc;
  // options
  int integrator, iterations, disableflags;
  float timestep, tolerance, pgs_scale, gravity[3];
  double timestep_d;  // time is accumulated in fp64 like mjData.time
  // bodies
  const int *body_parentid, *body_rootid, *body_jntnum, *body_jntadr, *body_dofnum, *body_dofadr,
      *body_subtree_end, *level_adr, *level_num, *level_body;
  const float *body_pos, *body_quat, *body_ipos, *body_iquat, *body_mass, *body_subtreemass,
      *body_inertia, *body_gravcomp, *body_invweight0;
  // joints / dofs
  const int *jnt_type, *jnt_qposadr, *jnt_dofadr, *jnt_bodyid, *jnt_actfrclimited;
  const float *jnt_pos, *jnt_axis, *jnt_stiffness, *jnt_range, *jnt_margin, *jnt_solref,
      *jnt_solimp, *jnt_actfrcrange;
  const int *dof_bodyid, *dof_jntid;
  const float *dof_armature, *dof_damping, *dof_frictionloss, *dof_solref, *dof_solimp,
      *dof_invweight0, *qpos0, *qpos_spring;
  const int* Mpair;  // [nMpair][2] (i, j) with j = i or an ancestor dof of i
  // geoms
  const int *geom_type, *geom_bodyid, *geom_group;
  const float *geom_size, *geom_pos, *geom_quat, *geom_rbound, *geom_rgba;
  // candidate collision pairs (static filters applied; g1 has the smaller geom type)
  const int *pair_g1, *pair_g2, *pair_dim;
  const float *pair_margin, *pair_gap, *pair_friction /*3*/, *pair_solref /*2*/, *pair_solimp /*5*/;
  // sites
  const int* site_bodyid;
  const float *site_pos, *site_quat;
  // cameras
  const int* cam_bodyid;
  const float *cam_pos, *cam_quat;
  // actuators (joint transmission)
  const int *act_dof, *act_qadr, *act_gaintype, *act_biastype, *act_ctrllimited, *act_forcelimited;
  const float *act_gear, *act_gainprm /*3*/, *act_biasprm /*3*/, *act_ctrlrange, *act_forcerange;
  // sensors
  const int *sensor_type, *sensor_objtype, *sensor_objid, *sensor_adr, *sensor_dim;
  const float* sensor_cutoff;
  const int *fric_dof, *lim_jnt, *rf_sensor;
};

// LDS layout of one environment (offsets in floats).  One wavefront owns one environment; the
// workgroup holds kEnvsPerBlock environments back to back.
struct LdsLayout {
  int xpos, xquat, xmat, xipos, xanchor, xaxis, gxpos, gxmat, scom, cinert, crb, cdof, cdofdot,
      cvel, cacc, cfrc, M, L, qpos, qvel, ctrl, qfrc_applied, qacc_ws, qfrc_bias, qfrc_passive,
      qfrc_act, qfrc_smooth, qacc_smooth, qacc, qfrc_con, act_force, Dg;
  int total;  // floats per env (multiple of 4)
};

// Per-env global scratch for constraint rows and contacts (offsets in floats within one env's
// region; the region of env e starts at e * total).
struct ScratchLayout {
  int efc_J, efc_MJ, efc_type, efc_pos, efc_margin, efc_floss, efc_R, efc_aref, efc_b, efc_f,
      efc_ARii, con;  // contact records: kConRec floats each
  int total;
};
constexpr int kConRec = 16;  // pair id (int bits), dist, pos[3], frame[9], pad[2]

constexpr int kEnvsPerBlock = 4;  // 256-thread workgroups, one wave per environment

// device state of a batch (all [n_envs][dim], fp32 unless noted)
struct DevState {
  float *qpos, *qvel, *ctrl, *qfrc_applied, *qacc_ws, *qacc, *qfrc_act, *sensordata;
  double* time;
  int* warning;  // [n_envs][4]
  int* ncon;     // [n_envs]
  float* scratch;
  float* geom_xpos;  // [n_envs][ngeom][3]  kinematics of the last forward (for the depth camera)
  float* geom_xmat;  // [n_envs][ngeom][9]
  float* cam_xpos;   // [n_envs][ncam][3]
  float* cam_xmat;   // [n_envs][ncam][9]
};

}  // namespace mrs
