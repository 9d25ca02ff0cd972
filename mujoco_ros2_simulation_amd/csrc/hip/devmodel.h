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

// Read-only model array.  On the device, element reads go through the AMDGPU constant address space
// (4): wave-uniform indices become scalar loads (s_load through the scalar cache), per-lane indices
// become global loads with an SGPR base.  Plain generic pointers loaded from a struct would compile to
// flat loads with 64-bit per-lane addresses.  Host code sees an ordinary pointer.
template <class T>
struct CPtr {
  const T* p;
  CPtr& operator=(const T* q) { p = q; return *this; }
  __device__ __forceinline__ T operator[](int i) const {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(4))) T*)p)[i];
#else
    return p[i];
#endif
  }
  __device__ __forceinline__ CPtr operator+(int i) const { return CPtr{p + i}; }
};

// LDS layout of one environment (offsets in floats).  One wavefront owns one environment; the
// workgroup holds 4*64/G environments back to back.
struct LdsLayout {
  int xpos, xquat, xmat, xipos, xanchor, xaxis, gxpos, gxmat, scom, cinert, crb, cdof, cdofdot,
      cvel, cacc, cfrc, M, L, qpos, qvel, ctrl, qfrc_applied, qacc_ws, qfrc_bias, qfrc_passive,
      qfrc_act, qfrc_smooth, qacc_smooth, qacc, qfrc_con, act_force,
      rfmask,  // per ray block: bitmask of candidate ray geoms (int bits)
      trees,   // blocked mode: per tree dofadr, dofnum, M block offset, pad (int bits)
      dofb,    // blocked mode: per dof its body and that body's subtree end (int bits; jac_col)
      H,       // blocked mode with a primal solver (Newton/CG): dense nv x nv Hessian and its factor
      Li,      // blocked mode with PGS: L^-1 per tree block (same offsets as L): the records' Y = L^-1 J'
      ten,     // fixed tendons: length and velocity per tendon of the step (smooth_forces)
      rk,      // RK4 models: the step's initial qpos [nq], then qvel [nv], stage velocity, B-weighted sums of
               // the stage velocities and accelerations [nv each]
      niter,   // constraint solver iterations of the last forward (int bits)
      hcon,    // helper waves: the step's contact and row counts from the helper (int bits)
      Lh;      // helper waves: the factor of M + h D for the integrator, built by the helper (0: none)
  int total;  // floats per env (multiple of 4)
};

// Per-env global scratch for constraint rows and contacts (offsets in floats within one env's
// region; the region of env e starts at e * total).
struct ScratchLayout {
  int efc_J, efc_MJ, efc_type, efc_pos, efc_margin, efc_floss, efc_R, efc_aref, efc_b, efc_f,
      efc_ARii, con, stage,  // contact records (kConRec floats each); per-lane narrow-phase staging
      efc_rec,               // blocked mode: row records in solver order (2 * pipe_w + 12 floats each)
      efc_rowof,             // blocked mode: row index of each record (int bits)
      efc_item,              // blocked mode: first row of the item starting at a record (int bits)
      efc_fq,                // blocked mode: row forces by record (global-record fallback path)
      efc_hdr,               // blocked mode: 8-float header of the item starting at a record
      efc_quad,              // blocked mode: per pipe, its first 16 items (record | rows << 16)
      efc_fd,                // elliptic models: the PGS row forces in fp64 (2 floats per row)
      sens,                  // sensordata sink of idle lane groups (envs past n_envs)
      efc_n;                 // rows of the dense layout of the last forward (int bits; -1: none stored)
  int total;
};
constexpr int kMaxPairCon = 8;  // contacts one geom pair can produce (box-box: the clipped face polygon)
constexpr int kConRec = 16;  // pair id (int bits), dist, pos[3], frame[9], first efc row (-1 if cut), first row (blocked mode)

// Everything the step kernel reads about the model.  Lives in device memory; the kernel receives
// one pointer to it.
struct DevModel {
  LdsLayout L;
  ScratchLayout S;
  // sizes
  int nq, nv, nu, nbody, njnt, ngeom, nsite, ncam, nsensor, nsensordata, max_depth, njump;
  int kin_onepass;  // every body has no joint or one hinge / free joint: kinematics' one-pass joint frames
  int fuse_ih;      // 16-lane implicitfast models: M + h D factored beside M (step.hip cholesky_ih)
  int nfric, nlim, npair, nrf, nMpair, max_con, max_efc, nrgeom, nrfblk, nsens_other, rf_common;
  // kinematic trees with dofs; blocked: M per tree + sparse constraint rows (set when G = 64);
  // pipe_w: dof slots per constraint row in the sparse solver (64 / pipe_w rows in flight per wave)
  int ntree, tree_nmax, nMblk, blocked, pipe_w;
  // sparse solver paths switched off (tests, A/B): bit 0 island-dual, bit 1 item-blocked, bit 2
  // register-resident (all off: the global-record solve); MRS_SPARSE_OFF
  int sparse_off;
  // workgroup-shared LDS tables (one copy per workgroup, after its envs' working sets; offsets in
  // floats from the start of the dynamic LDS): the ray-geom records (8 floats each) at shr_off, and
  // when rf_common the per-ray direction + sensordata address (4 floats each) at shr_off + shr_rf.
  // Staged once per launch, read by the ray phase every step instead of global loads.
  int shr_off, shr_rf, shr_total;
  // static ray split: when every rangefinder sits on a world-welded body, its hits on
  // world-welded geoms are the same every step and in every env.  rf_mode 1: the one-off producer
  // pass at batch creation, testing only those static geoms and writing the nearest hit per ray to
  // rf_static; rf_mode 2: the step kernel starts every ray from rf_static (staged in workgroup LDS
  // at shr_rfst) and tests only the moving geoms; 0: no split.  rf_static_mask: static ray-geom bits.
  int rf_mode, shr_rfst;
  // every rangefinder body is world-welded: rfblk frames and rfray origins / directions are stored
  // in the world frame (batch.hip), and the kernel uses them without the per-step body rotation
  int rf_static_frame;
  // the ray blocks' level-1 records (rfblk, 16 floats each, then the nrfblk slopes) at shr_blk, the
  // non-ray sensors' descriptors (sensrec, 16 floats each) at shr_sens
  int shr_blk, shr_sens;
  // friction-loss rows (fricrec: dof, R, B, frictionloss) at shr_fric, limited joints (limrec: qpos
  // address, margin, range) at shr_lim
  int shr_fric, shr_lim;
  // smooth-force tables (actrec, 20 floats per actuator; dofrec, 16 floats per dof) at shr_act, shr_dof
  int shr_act, shr_dof;
  // tree tables (bodytab, 8 floats per body; mpairtab, 4 floats per pair of M) at shr_body, shr_mpair
  int shr_body, shr_mpair;
  int shr_jump;  // the kinematics' pointer-jumping table (jump, int bits) with lane groups
  // kinematics tables (kinbody 25, kinjnt 13, kingeom 9 floats per entry; odd strides: lanes reading
  // consecutive entries hit distinct LDS banks) at shr_kbody, shr_kjnt, shr_kgeom with lane groups
  int shr_kbody, shr_kjnt, shr_kgeom;
  int shr_flag;  // helper waves: per physics wave (4 words) its count of com_pos passes this launch (int bits)
  unsigned rf_static_mask;
  float* rf_static;
  // options
  int integrator, iterations, disableflags, solver, ls_iterations;
  int restate;  // MRS_RESTATE_* (mrs_model.h): opt-in solver variants, 0 = upstream rules
  int cone;  // MRS_CONE_*: elliptic models take the dense row path (3-row contact blocks)
  int acc_sens;   // bit 0: accelerometer, bit 1: force/torque sensors present (mj_rnePostConstraint)
  int diag_skip;  // profiling ablation only (MRS_DIAG_SKIP); 0 in every measured/parity run
  float timestep, tolerance, pgs_scale, gravity[3], impratio, ls_tolerance;
  double timestep_d;  // time is accumulated in fp64 like mjData.time
  // bodies
  CPtr<int> body_parentid, body_rootid, body_jntnum, body_jntadr, body_dofnum, body_dofadr, body_subtree_end, level_adr, level_num, level_body;
  CPtr<int> jump;  // [njump][nbody]: ancestor at distance 2^r (-1 when that is the world or beyond)
  CPtr<float> body_pos, body_quat, body_ipos, body_iquat, body_mass, body_subtreemass, body_inertia, body_gravcomp, body_invweight0;
  // joints / dofs
  CPtr<int> jnt_type, jnt_qposadr, jnt_dofadr, jnt_bodyid, jnt_actfrclimited;
  CPtr<float> jnt_pos, jnt_axis, jnt_stiffness, jnt_range, jnt_margin, jnt_solref, jnt_solimp, jnt_actfrcrange;
  CPtr<int> dof_bodyid, dof_jntid;
  CPtr<float> dof_armature, dof_damping, dof_frictionloss, dof_solref, dof_solimp, dof_invweight0, qpos0, qpos_spring;
  CPtr<int> Mpair;  // [nMpair][2] (i, j) with j = i or an ancestor dof of i
  CPtr<int> body_tree, dof_tree, tree_dofadr, tree_dofnum, tree_Moff;  // tree -1: world / no dofs
  // geoms
  CPtr<int> geom_type, geom_bodyid, geom_group, geom_dataid;
  // mesh frames by triangle binning (batch.hip depth_kernel_mesh): the visible mesh geoms and the
  // first (geom, triangle) pair of each; nrast = 0 when the model has none (or exceeds its limits)
  CPtr<int> rast_geom, rast_base;
  int nrast, nrast_pair;
  CPtr<float> geom_size, geom_pos, geom_quat, geom_rbound, geom_rgba;
  // meshes (mrs_model.h): vertices in the mesh frame, triangles and convex-hull vertex ids (both
  // relative to the mesh's first vertex)
  CPtr<int> mesh_vertadr, mesh_faceadr, mesh_facenum, mesh_hulladr, mesh_hullnum, mesh_face, mesh_hull;
  // the hulls' faces as polygons (mrs_model.h mesh_poly*; step.hip poly_face_contacts)
  CPtr<int> mesh_polyadr, mesh_polynum, mesh_polyvertadr, mesh_polyvertnum, mesh_polyvert;
  CPtr<float> mesh_polynormal;
  CPtr<float> mesh_vert;
  // ray hierarchies (batch.hip build_mesh_bvh; mesh_face is reordered to their leaves): per mesh the
  // first node and the node count (0: none), 8 floats per node
  CPtr<int> mesh_bvhadr, mesh_bvhnum;
  CPtr<float> mesh_bvh;
  // the triangles pre-gathered in device face order (same index as mesh_face): vertex a and the edges
  // b - a, c - a in fp32, 9 floats each -- one load per triangle instead of face -> vertex chains
  CPtr<float> mesh_tri;
  // colour render: lit.h's packed light / material / texture block and each geom's material id
  CPtr<float> rlit;
  CPtr<int> geom_matid;
  int lit_nlight, lit_mat0, lit_tex0, lit_sky;
  // candidate collision pairs (static filters applied; g1 has the smaller geom type)
  // active equality constraints (mrs_model_view eq_*, inactive ones dropped on the host): neq of
  // them giving neq_rows rows (connect 3, weld 6, joint 1), first in the row order
  int neq, neq_rows;
  // fixed tendons (batch.hip): wraps, dense Jacobian rows ten_J [ntendon][nv], 12 constants per tendon
  // (stiffness, damping, lengthspring[2], range[2], margin, frictionloss, invweight0), the tendons
  // with friction-loss rows / limits, each actuator's tendon (-1: joint transmission); xrows: row
  // sources the blocked-mode sparse solver does not take (neq + nten_fric + nten_lim)
  int ntendon, nten_fric, nten_lim, xrows;
  CPtr<int> ten_adr, ten_num, wrap_qadr, wrap_dof, ten_fric, ten_lim, act_ten;
  CPtr<float> wrap_coef, ten_J, ten_prm, ten_solref_lim, ten_solimp_lim, ten_solref_fri, ten_solimp_fri;
  CPtr<int> eq_type, eq_obj1id, eq_obj2id;
  CPtr<float> eq_solref /*2*/, eq_solimp /*5*/, eq_data /*11*/;
  CPtr<int> pair_g1, pair_g2, pair_dim;
  CPtr<float> pair_margin, pair_gap, pair_friction /*3*/, pair_solref /*2*/, pair_solimp /*5*/;
  // sites
  CPtr<int> site_bodyid;
  CPtr<float> site_pos, site_quat;
  // cameras
  CPtr<int> cam_bodyid;
  CPtr<float> cam_pos, cam_quat;
  // actuators (joint transmission)
  CPtr<int> act_dof, act_qadr, act_gaintype, act_biastype, act_ctrllimited, act_forcelimited;
  CPtr<float> act_gear, act_gainprm /*3*/, act_biasprm /*3*/, act_ctrlrange, act_forcerange;
  // sensors
  CPtr<int> sensor_type, sensor_objtype, sensor_objid, sensor_adr, sensor_dim;
  CPtr<float> sensor_cutoff;
  CPtr<int> fric_dof, lim_jnt, rf_sensor, sens_other;  // sens_other: non-rangefinder sensor ids
  CPtr<float> sensrec;  // their descriptors (batch.hip), 16 floats each
  CPtr<float> fricrec, limrec;  // 4 floats per friction-loss dof / limited joint (batch.hip)
  CPtr<float> actrec, dofrec;   // smooth-force tables (batch.hip)
  CPtr<float> bodytab, mpairtab;  // tree tables of the smooth dynamics (batch.hip)
  CPtr<float> kinbody, kinjnt, kingeom;  // kinematics tables (batch.hip; step.hip kin_body / kin_jnt / kin_geom)
  // ray-visible geoms (rgba alpha != 0, what mj_ray tests), packed 8 floats per geom so one wide
  // scalar load fetches a record: geom id, type, body (int bits), rbound, size[3], pad
  CPtr<float> rgeom;
  // ray blocks of kRayBlock consecutive rangefinders, 16 floats each: body, fan flag (int bits),
  // origin[3], axis a[3], in-plane b[3], normal c[3] in the body frame, cos and sin of the in-plane
  // half-angle; followed by nrfblk out-of-plane slopes eps.  rf_common: all blocks are fans from
  // one point of one body
  CPtr<float> rfblk;
  // per rangefinder, 8 floats: unit direction[3], sensordata address (int bits), body (int bits),
  // origin[3], in the body frame
  CPtr<float> rfray;
};
constexpr int kRayBlock = 128;

// waves per workgroup: 256-thread workgroups with lane groups (G < 64); one wave (one env) per
// workgroup at G = 64, so LDS is granted per env (the C5 working set of ~13.5 KB fits 11 envs per
// CU instead of 2 workgroups of 4)
template <int G>
#ifndef MRS_G16_WAVES
#define MRS_G16_WAVES 4
#endif
struct WavesPerBlock { static constexpr int value = G == 64 ? 1 : (G == 16 ? MRS_G16_WAVES : 4); };
// environments per workgroup of the step kernel at group width g (kEnvsPerBlock); G = 16 kernels
// take their waves per workgroup at run time (DevState::wpb16, at most WavesPerBlock<16>)
inline int envs_per_block(int g, int wpb16 = WavesPerBlock<16>::value) {
  switch (g) {
    case 8: return WavesPerBlock<8>::value * 8;
    case 16: return wpb16 * 4;
    case 32: return WavesPerBlock<32>::value * 2;
    default: return WavesPerBlock<64>::value;
  }
}

// device state of a batch (all [n_envs][dim], fp32 unless noted)
struct DevState {
  float *qpos, *qvel, *ctrl, *qfrc_applied, *qacc_ws, *qacc, *qfrc_act, *sensordata;
  double* time;
  int* warning;  // [n_envs][4]
  int* ncon;     // [n_envs]
  int* niter;    // [n_envs] constraint solver iterations of the last step (mjData.solver_niter)
  float* scratch;
  float* geom_xpos;  // [n_envs][ngeom][3]  kinematics of the last forward (for the depth camera)
  float* geom_xmat;  // [n_envs][ngeom][9]
  float* cam_xpos;   // [n_envs][ncam][3]
  float* cam_xmat;   // [n_envs][ncam][9]
  // env spread (occupancy for small batches): 2^spread_shift lane groups step each env, the first
  // (primary) writes the results, the others mirror it in their own scratch (slot scr_mirror + group);
  // a batch of few envs then spreads over more waves / SIMDs.  0 = one group per env.
  int spread_shift, scr_mirror;
  // waves per workgroup of the G = 16 kernels (1 .. WavesPerBlock<16>): one-wave workgroups when the
  // batch has fewer waves than the device has SIMDs, so they spread over every CU (batch_create)
  int wpb16;
  // 1: G = 16 step launches add a ray helper wave per physics wave (step_kernel; batch_create)
  int ray_helpers;
};

}  // namespace mrs
