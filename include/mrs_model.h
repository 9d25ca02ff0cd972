/*
 * mrs_model.h — flat, read-only view of a compiled MJCF model.
 *
 * This is the compiled-model contract shared by the product (the HIP step kernels, which pack it
 * into a device constant block) and by the test oracle under oracle/ (which steps it on the CPU in
 * fp64).  It plays the role of MuJoCo's mjModel for the subset of fields the hot path needs; field
 * names follow mjModel so a maintainer can map them one-to-one.  The reference reads these mjModel
 * fields directly (SURVEY.md §2 "mjModel fields read by the plugin"):
 *   nq, nv, nu, nsensor, nsensordata, ncam            src/mujoco_system_interface.cpp:1193-1213
 *   jnt_type, jnt_qposadr, jnt_dofadr                 src/mujoco_system_interface.cpp:1223-1226
 *   actuator_trntype/trnid/biastype/biasprm           src/mujoco_system_interface.cpp:433-460,1200-1206
 *   sensor_type, sensor_adr                           src/mujoco_lidar.cpp:130-200
 *   cam_resolution, cam_fovy                          src/mujoco_cameras.cpp:45-47
 *   vis.map.znear/zfar, stat.extent                   src/mujoco_cameras.cpp:222-223
 *
 * All arrays are owned by the model object that produced the view (mrs_model_view()).
 * Layout: row-major, per-object blocks, doubles for reals (the model is compiled in fp64; the GPU
 * packs a float32 copy).
 */
#ifndef MRS_MODEL_H
#define MRS_MODEL_H

#ifdef __cplusplus
extern "C" {
#endif

/* enum values follow MuJoCo 3.3 (mjtGeom, mjtJoint, mjtIntegrator, mjtSolver, mjtTrn, mjtGain,
 * mjtBias, mjtDyn).  Sensor types are this project's own numbering (names match mjtSensor). */
enum { MRS_GEOM_PLANE = 0, MRS_GEOM_HFIELD = 1, MRS_GEOM_SPHERE = 2, MRS_GEOM_CAPSULE = 3,
       MRS_GEOM_ELLIPSOID = 4, MRS_GEOM_CYLINDER = 5, MRS_GEOM_BOX = 6, MRS_GEOM_MESH = 7 };
enum { MRS_JNT_FREE = 0, MRS_JNT_BALL = 1, MRS_JNT_SLIDE = 2, MRS_JNT_HINGE = 3 };
enum { MRS_INT_EULER = 0, MRS_INT_RK4 = 1, MRS_INT_IMPLICIT = 2, MRS_INT_IMPLICITFAST = 3 };
enum { MRS_SOL_PGS = 0, MRS_SOL_CG = 1, MRS_SOL_NEWTON = 2 };
enum { MRS_CONE_PYRAMIDAL = 0, MRS_CONE_ELLIPTIC = 1 };  /* mjtCone */
enum { MRS_EQ_CONNECT = 0, MRS_EQ_WELD = 1, MRS_EQ_JOINT = 2 };  /* mjtEq subset */
enum { MRS_TEX_2D = 0, MRS_TEX_CUBE = 1, MRS_TEX_SKYBOX = 2 };  /* mjtTexture */
enum { MRS_BUILTIN_NONE = 0, MRS_BUILTIN_GRADIENT = 1, MRS_BUILTIN_CHECKER = 2, MRS_BUILTIN_FLAT = 3 };
enum { MRS_MARK_NONE = 0, MRS_MARK_EDGE = 1, MRS_MARK_CROSS = 2 };
#define MRS_NEQDATA 11
enum { MRS_TRN_JOINT = 0, MRS_TRN_TENDON = 3 };
enum { MRS_DYN_NONE = 0 };
enum { MRS_GAIN_FIXED = 0, MRS_GAIN_AFFINE = 1 };
enum { MRS_BIAS_NONE = 0, MRS_BIAS_AFFINE = 1 };
enum { MRS_OBJ_UNKNOWN = 0, MRS_OBJ_BODY = 1, MRS_OBJ_JOINT = 3, MRS_OBJ_GEOM = 5, MRS_OBJ_SITE = 6,
       MRS_OBJ_CAMERA = 7, MRS_OBJ_MESH = 10, MRS_OBJ_TENDON = 18, MRS_OBJ_ACTUATOR = 19, MRS_OBJ_SENSOR = 20 };
enum { MRS_SENS_ACCELEROMETER = 1, MRS_SENS_GYRO = 3, MRS_SENS_FORCE = 4, MRS_SENS_TORQUE = 5,
       MRS_SENS_RANGEFINDER = 7, MRS_SENS_JOINTPOS = 9, MRS_SENS_JOINTVEL = 10,
       MRS_SENS_ACTUATORFRC = 15, MRS_SENS_FRAMEPOS = 25, MRS_SENS_FRAMEQUAT = 26 };
/* restate bits (not MuJoCo options; mrs_model_set_restate): opt-in variants of this restatement that
 * upstream does not have.  NEWTON_REFINE: after a Newton step that kept every row's state, one more
 * step from freshly formed residuals with the same factor, then stop (mj_solNewton instead keeps
 * iterating until its improvement / gradient tests stop it).  PGS_ELLIPTIC_BLOCK: PGS solves each
 * elliptic contact block exactly over its cone (mj_solPGS takes a normal / ray step, then the friction
 * by mju_QCQP2 with the normal fixed). */
enum { MRS_RESTATE_NEWTON_REFINE = 1 << 0, MRS_RESTATE_PGS_ELLIPTIC_BLOCK = 1 << 1,
       MRS_RESTATE_NO_MPR_POLISH = 1 << 2, /* diagnostics: keep MPR's own contact (no normal polish) */
       MRS_RESTATE_NO_MULTICCD = 1 << 3 /* diagnostics: one MPR contact for face-on polytope pairs too */ };
/* disable flags (mjtDisableBit subset) */
enum { MRS_DSBL_CONSTRAINT = 1 << 0, MRS_DSBL_EQUALITY = 1 << 1, MRS_DSBL_FRICTIONLOSS = 1 << 2,
       MRS_DSBL_LIMIT = 1 << 3, MRS_DSBL_CONTACT = 1 << 4, MRS_DSBL_PASSIVE = 1 << 5,
       MRS_DSBL_GRAVITY = 1 << 6, MRS_DSBL_CLAMPCTRL = 1 << 7, MRS_DSBL_WARMSTART = 1 << 8,
       MRS_DSBL_FILTERPARENT = 1 << 9, MRS_DSBL_ACTUATION = 1 << 10, MRS_DSBL_REFSAFE = 1 << 11,
       MRS_DSBL_SENSOR = 1 << 12, MRS_DSBL_EULERDAMP = 1 << 15, MRS_DSBL_AUTORESET = 1 << 16 };

#define MRS_NGAIN 10
#define MRS_NBIAS 10
#define MRS_NREF 2
#define MRS_NIMP 5

typedef struct mrs_model_view {
  /* sizes */
  int nq, nv, nu, na, nbody, njnt, ngeom, nsite, ncam, nsensor, nsensordata, nkey;
  int nM;            /* nv*nv (dense joint-space matrices on this path) */
  int max_depth;     /* longest root-to-leaf body chain (levels for tree-parallel passes) */
  int npair;         /* statically admissible collision pairs (broad-phase filters of mj_collision) */

  /* options (mjOption subset) */
  double timestep, gravity[3], tolerance, impratio, ls_tolerance;
  int integrator, solver, iterations, disableflags, cone, ls_iterations;
  int restate;       /* MRS_RESTATE_* bits: this build's own solver variants (0 = the upstream rules) */

  /* statistic / visual (for the depth camera) */
  double stat_extent, stat_center[3], stat_meaninertia, vis_znear, vis_zfar;

  /* bodies: world is body 0 */
  const int *body_parentid, *body_rootid, *body_weldid, *body_jntnum, *body_jntadr, *body_dofnum,
      *body_dofadr, *body_geomnum, *body_geomadr, *body_depth;
  const double *body_pos /*3*/, *body_quat /*4*/, *body_ipos /*3*/, *body_iquat /*4*/,
      *body_mass, *body_subtreemass, *body_inertia /*3*/, *body_invweight0 /*2*/, *body_gravcomp;

  /* joints */
  const int *jnt_type, *jnt_qposadr, *jnt_dofadr, *jnt_bodyid, *jnt_limited, *jnt_actfrclimited;
  const double *jnt_pos /*3*/, *jnt_axis /*3*/, *jnt_stiffness, *jnt_range /*2*/,
      *jnt_actfrcrange /*2*/, *jnt_margin, *jnt_solref /*2*/, *jnt_solimp /*5*/;

  /* dofs */
  const int *dof_bodyid, *dof_jntid, *dof_parentid;
  const double *dof_armature, *dof_damping, *dof_frictionloss, *dof_solref /*2*/,
      *dof_solimp /*5*/, *dof_invweight0, *dof_M0;

  /* geoms */
  const int *geom_type, *geom_contype, *geom_conaffinity, *geom_condim, *geom_bodyid, *geom_group,
      *geom_priority;
  const double *geom_size /*3*/, *geom_pos /*3*/, *geom_quat /*4*/, *geom_rbound,
      *geom_friction /*3*/, *geom_margin, *geom_gap, *geom_solmix, *geom_solref /*2*/,
      *geom_solimp /*5*/, *geom_rgba /*4*/;

  /* sites */
  const int *site_bodyid;
  const double *site_pos /*3*/, *site_quat /*4*/;

  /* cameras */
  const int *cam_bodyid, *cam_resolution /*2*/;
  const double *cam_pos /*3*/, *cam_quat /*4*/, *cam_fovy;

  /* actuators */
  const int *actuator_trntype, *actuator_dyntype, *actuator_gaintype, *actuator_biastype,
      *actuator_trnid /*2*/, *actuator_ctrllimited, *actuator_forcelimited;
  const double *actuator_gear /*6*/, *actuator_gainprm /*10*/, *actuator_biasprm /*10*/,
      *actuator_ctrlrange /*2*/, *actuator_forcerange /*2*/;

  /* sensors */
  const int *sensor_type, *sensor_objtype, *sensor_objid, *sensor_dim, *sensor_adr;
  const double *sensor_cutoff;

  /* default configuration */
  const double *qpos0, *qpos_spring;

  /* keyframes */
  const double *key_time, *key_qpos, *key_qvel, *key_ctrl;

  /* candidate collision pairs [npair]: geoms of different weld groups, not parent-child welds,
   * contype/conaffinity compatible; the lower geom type first */
  const int *pair_geom1, *pair_geom2;

  /* meshes (mjModel mesh_*): vertices [nmeshvert][3] in the mesh's inertial frame (MuJoCo recentres
   * a mesh at its centre of mass and aligns it with its principal axes; geom_pos/geom_quat carry
   * the offset), triangles [nmeshface][3] (vertex ids relative to mesh_vertadr), convex-hull vertex
   * ids [nmeshhull] (relative to mesh_vertadr) used by collision; geom_dataid = mesh id or -1 */
  int nmesh, nmeshvert, nmeshface, nmeshhull;
  const int *geom_dataid, *mesh_vertadr, *mesh_vertnum, *mesh_faceadr, *mesh_facenum, *mesh_hulladr,
      *mesh_hullnum, *mesh_face, *mesh_hull;
  const double *mesh_vert;

  /* explicit <contact><pair> (mjModel npair / pair_*): collided before the candidate pairs above,
   * whatever contype/conaffinity and the body filters say, with their own parameters (attributes the
   * pair omits are mixed from its geoms as for candidate pairs); geom1 has the lower type.  And
   * <contact><exclude> body pairs (mjModel exclude_signature), which -- like the bodies of an
   * explicit pair -- the candidate list above already leaves out. */
  int nexpair, nexclude;
  const int *expair_geom1, *expair_geom2, *expair_dim, *exclude_body1, *exclude_body2;
  const double *expair_friction /*5*/, *expair_solref /*2*/, *expair_solimp /*5*/, *expair_margin, *expair_gap;

  /* equality constraints (mjModel neq / eq_*; MRS_EQ_*): obj1 / obj2 are bodies (connect, weld; obj2
   * 0 = world) or joints (joint; obj2 -1 = none).  eq_data [neq][11]:
   *   connect: anchor in body1's frame (0:3), the same point in body2's frame at qpos0 (3:6);
   *   weld:    anchor in body2's frame (0:3), body2's pose in body1's frame: pos (3:6), quat (6:10),
   *            torquescale (10);
   *   joint:   polycoef (0:5), then qpos0 of joint1 (5) and joint2 (6). */
  int neq;
  const int *eq_type, *eq_obj1id, *eq_obj2id, *eq_active0;
  const double *eq_solref /*2*/, *eq_solimp /*5*/, *eq_data /*11*/;

  /* rendering (mjModel light_* / tex_* / mat_*, mjVisual headlight): the camera colour image's
   * restatement of MuJoCo's OpenGL lighting.  Lights are fixed in the world (on the
   * world body or a body welded to it; pos / dir world frame); textures are MuJoCo's procedural
   * builtins (MRS_TEX_*: checker / gradient / flat, marks none / edge / cross), 2-D or skybox;
   * geom_matid -1 = no material (rgba only). */
  double vis_headlight[10];  /* ambient[3], diffuse[3], specular[3], active */
  int nlight, ntex, nmat;
  const int *light_directional, *light_castshadow, *light_active, *tex_type, *tex_builtin, *tex_mark,
      *tex_width, *tex_height, *mat_texid, *mat_texuniform, *geom_matid;
  const double *light_pos /*3*/, *light_dir /*3*/, *light_ambient /*3*/, *light_diffuse /*3*/,
      *light_specular /*3*/, *light_attenuation /*3*/, *light_cutoff, *light_exponent, *tex_rgb1 /*3*/,
      *tex_rgb2 /*3*/, *tex_markrgb /*3*/, *mat_rgba /*4*/, *mat_texrepeat /*2*/, *mat_specular,
      *mat_shininess, *mat_emission;

  /* fixed tendons (mjModel ntendon / tendon_* / wrap_*, mjTRN_TENDON actuators): tendon t is the linear
   * combination length = sum_k wrap_prm[k] qpos[jnt_qposadr[wrap_objid[k]]] over its wraps
   * k in [tendon_adr[t], tendon_adr[t] + tendon_num[t]) of hinge / slide joints; ten_J is constant.
   * Spring force -stiffness (length - lengthspring) outside the dead band [lengthspring[0],
   * lengthspring[1]], damping -damping * velocity, limit rows on [range[0], range[1]] within margin,
   * a friction-loss row when frictionloss > 0; diagApprox tendon_invweight0 = J M(qpos0)^-1 J'. */
  int ntendon, nwrap;
  const int *tendon_adr, *tendon_num, *tendon_limited, *wrap_objid;
  const double *wrap_prm, *tendon_range /*2*/, *tendon_margin, *tendon_solref_lim /*2*/,
      *tendon_solimp_lim /*5*/, *tendon_frictionloss, *tendon_solref_fri /*2*/, *tendon_solimp_fri /*5*/,
      *tendon_stiffness, *tendon_damping, *tendon_lengthspring /*2*/, *tendon_invweight0, *tendon_length0;

  /* the meshes' convex-hull faces as polygons (coplanar hull triangles merged; collision's face
   * contacts): mesh k's polygons are [mesh_polyadr[k], + mesh_polynum[k]); polygon p
   * has the outward unit normal mesh_polynormal[p] (mesh frame) and the vertex ids (relative to
   * mesh_vertadr) mesh_polyvert[mesh_polyvertadr[p] .. + mesh_polyvertnum[p]), counter-clockwise
   * about the normal */
  int nmeshpoly, nmeshpolyvert;
  const int *mesh_polyadr, *mesh_polynum, *mesh_polyvertadr, *mesh_polyvertnum, *mesh_polyvert;
  const double *mesh_polynormal /*3*/;
} mrs_model_view;

#ifdef __cplusplus
}
#endif
#endif /* MRS_MODEL_H */
