/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.  fp64 CPU restatement of the MuJoCo 3.3.4 mj_step subset
 * on this repo's hot path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product never links it.
 *
 * Parity status: MuJoCo itself is third-party, not vendored in /root/reference and not installable
 * here, so this restatement follows MuJoCo's published algorithms (engine_forward,
 * engine_core_smooth, engine_core_constraint, engine_solver, engine_ray, engine_collision_*) as
 * documented for 3.3.4, and is pinned by closed-form known answers (tests/test_oracle_kat.py: mass
 * matrix of the reference's 2-DoF arm, dampratio->kv, the reference scene's 24 lidar ranges, a
 * 1-DoF servo recurrence, ballistic flight, depth of a plane) and by the reference's own
 * behavioural pin (test/src/robot_launch_test.py:112-132: joints within 0.05 rad of [0.5,-0.5]
 * after 2 s).  Against upstream mj_step it is "parity unpinned" beyond those pins.
 */
#ifndef MRS_ORACLE_H
#define MRS_ORACLE_H

#include "../include/mrs_model.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_data {
  /* state and inputs (mjData names) */
  double *qpos, *qvel, *ctrl, *qfrc_applied, *qacc_warmstart;
  double time;
  /* outputs of the last step/forward */
  double *qacc, *qfrc_actuator, *sensordata;
  int warning[4]; /* bad qpos count, bad qvel count, bad qacc count, last info */
  int ncon, nefc;
  int solver_niter; /* PGS sweeps of the last step */
  void* ws;       /* private workspace */
} orc_data;

orc_data* orc_make_data(const mrs_model_view* m);
void orc_free_data(orc_data* d);
void orc_reset(const mrs_model_view* m, orc_data* d, int key);
void orc_step(const mrs_model_view* m, orc_data* d);
void orc_forward(const mrs_model_view* m, orc_data* d);

/* introspection for tests: dense joint-space inertia at the current qpos (nv*nv) */
void orc_mass_matrix(const mrs_model_view* m, orc_data* d, double* M);
/* d qfrc_bias / d qvel at the current state after a forward (nv*nv, row i = bias component i): the
 * RNE velocity derivative the full implicit integrator adds to its matrix */
void orc_bias_vel(const mrs_model_view* m, orc_data* d, double* dB);
/* kinematics at the current qpos: body xpos (nbody*3), xquat (nbody*4), geom xpos (ngeom*3),
 * geom xmat (ngeom*9); any pointer may be NULL */
void orc_kinematics(const mrs_model_view* m, orc_data* d, double* xpos, double* xquat,
                    double* geom_xpos, double* geom_xmat);
/* mj_ray against the geoms of the current kinematics (call orc_kinematics/forward first) */
double orc_ray(const mrs_model_view* m, orc_data* d, const double pnt[3], const double vec[3],
               int bodyexclude, int* geomid);
/* depth image (H*W floats, ROS row order, eye-space z, `far` on miss) of camera `cam` */
void orc_render_depth(const mrs_model_view* m, orc_data* d, int cam, float* out);
/* depth (may be NULL) and RGB8 [H][W][3] of camera `cam`: flat headlight shading of each pixel's
 * nearest geom, black on a miss (the device's mrs_batch_render_rgbd) */
void orc_render_rgbd(const mrs_model_view* m, orc_data* d, int cam, float* depth, unsigned char* rgb);
/* contacts of the last forward: up to `max` records of {geom1, geom2, dist, pos[3], frame[9]} */
int orc_efc(orc_data* d, int nv, int max, int* type, double* force, double* aref, double* R, double* pos,
            double* J);
int orc_contacts(orc_data* d, int max, int* geom, double* dist, double* pos, double* frame);
/* statically admissible collision pairs by the oracle's own filter (lower geom type first); returns
 * the count, writes up to `max` */
int orc_candidate_pairs(const mrs_model_view* m, int max, int* geom1, int* geom2);
/* qacc_smooth, qfrc_smooth (nv each) of the last forward */
void orc_smooth(const mrs_model_view* m, orc_data* d, double* qacc_smooth, double* qfrc_smooth);

/* CPU baseline: step `n_envs` independent copies `n_steps` times with ctrl held per period of
 * `period` steps; ctrl_table is [n_periods][n_envs][nu], qpos_init [n_envs][nq].  Runs on
 * `n_threads` pthreads (one env per task).  Returns wall seconds; final qpos/qvel written out. */
double orc_rollout(const mrs_model_view* m, int n_envs, int n_steps, int period,
                   const double* ctrl_table, const double* qpos_init, int n_threads,
                   double* qpos_out, double* qvel_out);

#ifdef __cplusplus
}
#endif
#endif
