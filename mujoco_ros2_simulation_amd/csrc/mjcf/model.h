// Compiled model (host side).  Owns the arrays behind mrs_model_view (include/mrs_model.h) plus
// names.  Produced by compile_mjcf(); plays the role of mjModel for the subset on the hot path.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "../../../include/mrs_model.h"

namespace mrs {

struct Model {
  int nq = 0, nv = 0, nu = 0, na = 0, nbody = 0, njnt = 0, ngeom = 0, nsite = 0, ncam = 0,
      nsensor = 0, nsensordata = 0, nkey = 0, max_depth = 0;

  double timestep = 0.002, gravity[3] = {0, 0, -9.81}, tolerance = 1e-8, impratio = 1,
         ls_tolerance = 0.01;
  int integrator = MRS_INT_EULER, solver = MRS_SOL_NEWTON, iterations = 100, disableflags = 0,
      cone = 0, ls_iterations = 50, restate = 0;

  double stat_extent = 0, stat_center[3] = {0, 0, 0}, stat_meaninertia = 1, vis_znear = 0.01,
         vis_zfar = 50;

  std::vector<int> body_parentid, body_rootid, body_weldid, body_jntnum, body_jntadr, body_dofnum,
      body_dofadr, body_geomnum, body_geomadr, body_depth;
  std::vector<double> body_pos, body_quat, body_ipos, body_iquat, body_mass, body_subtreemass,
      body_inertia, body_invweight0, body_gravcomp;

  std::vector<int> jnt_type, jnt_qposadr, jnt_dofadr, jnt_bodyid, jnt_limited, jnt_actfrclimited;
  std::vector<double> jnt_pos, jnt_axis, jnt_stiffness, jnt_range, jnt_actfrcrange, jnt_margin,
      jnt_solref, jnt_solimp;

  std::vector<int> dof_bodyid, dof_jntid, dof_parentid;
  std::vector<double> dof_armature, dof_damping, dof_frictionloss, dof_solref, dof_solimp,
      dof_invweight0, dof_M0;

  std::vector<int> geom_type, geom_contype, geom_conaffinity, geom_condim, geom_bodyid, geom_group,
      geom_priority;
  std::vector<double> geom_size, geom_pos, geom_quat, geom_rbound, geom_friction, geom_margin,
      geom_gap, geom_solmix, geom_solref, geom_solimp, geom_rgba;

  std::vector<int> site_bodyid;
  std::vector<double> site_pos, site_quat;

  std::vector<int> cam_bodyid, cam_resolution;
  std::vector<double> cam_pos, cam_quat, cam_fovy;

  std::vector<int> actuator_trntype, actuator_dyntype, actuator_gaintype, actuator_biastype,
      actuator_trnid, actuator_ctrllimited, actuator_forcelimited;
  std::vector<double> actuator_gear, actuator_gainprm, actuator_biasprm, actuator_ctrlrange,
      actuator_forcerange;

  std::vector<int> sensor_type, sensor_objtype, sensor_objid, sensor_dim, sensor_adr;
  std::vector<double> sensor_cutoff;

  std::vector<double> qpos0, qpos_spring;
  std::vector<double> key_time, key_qpos, key_qvel, key_ctrl;
  // meshes: vertices in the mesh's inertial frame (centre of mass, principal axes), triangles, and the
  // convex hull's vertex ids (relative to the mesh's first vertex); geom_dataid = mesh id or -1
  int nmesh = 0;
  std::vector<int> geom_dataid, mesh_vertadr, mesh_vertnum, mesh_faceadr, mesh_facenum, mesh_hulladr,
      mesh_hullnum, mesh_face, mesh_hull;
  // hull faces as polygons (mrs_model.h): per mesh polyadr / polynum; per polygon the vertex-list
  // address and length (mesh_polynum_v) and its outward normal; the vertex ids
  std::vector<int> mesh_polyadr, mesh_polynum, mesh_polyvertadr, mesh_polynum_v, mesh_polyvert;
  std::vector<double> mesh_polynormal;
  std::vector<double> mesh_vert;
  // statically admissible collision pairs (mj_collision's broad-phase filters), lower geom type first
  std::vector<int> pair_geom1, pair_geom2;
  // explicit <contact><pair> (own parameters) and <contact><exclude> body pairs (mrs_model_view)
  std::vector<int> expair_geom1, expair_geom2, expair_dim, exclude_body1, exclude_body2;
  std::vector<double> expair_friction, expair_solref, expair_solimp, expair_margin, expair_gap;
  // equality constraints (mrs_model_view eq_*)
  std::vector<int> eq_type, eq_obj1id, eq_obj2id, eq_active0;
  std::vector<double> eq_solref, eq_solimp, eq_data;
  // fixed tendons (mrs_model_view tendon_* / wrap_*)
  std::vector<int> tendon_adr, tendon_num, tendon_limited, wrap_objid;
  std::vector<double> wrap_prm, tendon_range, tendon_margin, tendon_solref_lim, tendon_solimp_lim,
      tendon_frictionloss, tendon_solref_fri, tendon_solimp_fri, tendon_stiffness, tendon_damping,
      tendon_lengthspring, tendon_invweight0, tendon_length0;
  // rendering (mrs_model_view light_* / tex_* / mat_*); MuJoCo's headlight defaults
  double vis_headlight[10] = {0.1, 0.1, 0.1, 0.4, 0.4, 0.4, 0.5, 0.5, 0.5, 1};
  std::vector<int> light_directional, light_castshadow, light_active, tex_type, tex_builtin, tex_mark, tex_width,
      tex_height, mat_texid, mat_texuniform, geom_matid;
  std::vector<double> light_pos, light_dir, light_ambient, light_diffuse, light_specular, light_attenuation,
      light_cutoff, light_exponent, tex_rgb1, tex_rgb2, tex_markrgb, mat_rgba, mat_texrepeat, mat_specular,
      mat_shininess, mat_emission;

  // names per object type (MRS_OBJ_*), index = object id
  std::map<int, std::vector<std::string>> names;
  std::string model_name;

  int name2id(int objtype, const std::string& name) const;
  const char* id2name(int objtype, int id) const;
  mrs_model_view view() const;
};

// Compile an MJCF file (path) or string (xml + base directory for <include>).  Throws
// std::runtime_error with a message on any unsupported or malformed input.
Model compile_mjcf_file(const std::string& path);
Model compile_mjcf_string(const std::string& xml, const std::string& basedir);

}  // namespace mrs
