/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h).  fp64 scalar CPU restatement of the
 * MuJoCo 3.3.4 mj_step pipeline subset used by this repo's hot path.  One environment per call;
 * orc_rollout() threads over environments for the CPU baseline.
 *
 * Reference anchors: the plugin calls this pipeline through mj_step at
 * src/mujoco_system_interface.cpp:1691,1731 and mj_forward at :741,1771; rangefinder sensordata is
 * consumed at src/mujoco_lidar.cpp:249; the depth image at src/mujoco_cameras.cpp:214-240.
 * Upstream stage names are given on each function ([upstream] = MuJoCo 3.3.4 source layout).
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#define MINVAL 1e-15
#define MAXVAL 1e10
#define MAXCON 256
#define MAXEFC 1024

typedef struct {
  int geom[2];
  double dist, pos[3], frame[9], friction[3], solref[2], solimp[5], includemargin;
  int dim;
} orc_contact;

typedef struct {
  /* kinematics */
  double *xpos, *xquat, *xmat, *xipos, *ximat, *xanchor, *xaxis, *geom_xpos, *geom_xmat;
  double *subtree_com, *cinert, *cdof, *crb, *cvel, *cdof_dot, *cacc, *cfrc;
  double *cacc_full, *cfrc_ext, *cfrc_int; /* mj_rnePostConstraint outputs */
  int efc_con_first[MAXCON];              /* first efc row of each contact */
  /* dynamics */
  double *M, *L, *qfrc_bias, *qfrc_passive, *qfrc_smooth, *qacc_smooth, *qfrc_constraint,
      *actuator_force, *tmp, *tmp2, *Mi, *Li;
  /* constraints */
  int nefc, ncon;
  int efc_type[MAXEFC], efc_id[MAXEFC];
  double *efc_J, *efc_MinvJT;
  double efc_pos[MAXEFC], efc_margin[MAXEFC], efc_frictionloss[MAXEFC], efc_diag[MAXEFC],
      efc_R[MAXEFC], efc_D[MAXEFC], efc_aref[MAXEFC], efc_b[MAXEFC], efc_force[MAXEFC],
      efc_vel[MAXEFC], efc_solref[MAXEFC][2], efc_solimp[MAXEFC][5], efc_KBIP[MAXEFC][4],
      efc_rscale[MAXEFC], efc_jar[MAXEFC], efc_jv[MAXEFC];
  int efc_state[MAXEFC];
  /* elliptic cones: row k of its contact's block (0 normal, 1-2 tangents; -1 for every other row),
   * the block's regularised cone mu = friction / sqrt(impratio) and the tangents' friction coefficient */
  int efc_sub[MAXEFC];
  double efc_mu[MAXEFC], efc_fr[MAXEFC];
  double* AR;
  orc_contact con[MAXCON];
} orc_ws;

enum { EFC_FRICTION = 1, EFC_LIMIT = 2, EFC_CONTACT = 3, EFC_EQUALITY = 4, EFC_TFRICTION = 5, EFC_TLIMIT = 6 };
/* equality rows are unbounded; the solvers treat them as friction-loss rows with this bound (never
 * reached: a force of 1e15), so they are quadratic in every primal state and unclamped in PGS */
#define EQ_BOUND 1e15
#define FRIC_LIKE(t) ((t) == EFC_FRICTION || (t) == EFC_EQUALITY || (t) == EFC_TFRICTION)
/* an elliptic contact block starts at row r (its normal) */
#define ELL_BLOCK(w, r) ((w)->efc_sub[r] == 0)

/* ------------------------------------------------------------------------ small math */
static void quat_mul(double r[4], const double a[4], const double b[4]) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof t);
}
static void quat_normalize(double q[4]) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}
static void quat2mat(double m[9], const double q[4]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = w * w + x * x - y * y - z * z; m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = w * w - x * x + y * y - z * z; m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = w * w - x * x - y * y + z * z;
}
static void mat_vec(double r[3], const double m[9], const double v[3]) {
  double t[3] = {m[0] * v[0] + m[1] * v[1] + m[2] * v[2], m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
                 m[6] * v[0] + m[7] * v[1] + m[8] * v[2]};
  memcpy(r, t, sizeof t);
}
static void matT_vec(double r[3], const double m[9], const double v[3]) {
  double t[3] = {m[0] * v[0] + m[3] * v[1] + m[6] * v[2], m[1] * v[0] + m[4] * v[1] + m[7] * v[2],
                 m[2] * v[0] + m[5] * v[1] + m[8] * v[2]};
  memcpy(r, t, sizeof t);
}
static void rot_quat(double r[3], const double v[3], const double q[4]) {
  double m[9];
  quat2mat(m, q);
  mat_vec(r, m, v);
}
static void cross3(double r[3], const double a[3], const double b[3]) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  memcpy(r, t, sizeof t);
}
static double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double norm3(const double a[3]) { return sqrt(dot3(a, a)); }
static double normalize3(double a[3]) {
  double n = norm3(a);
  if (n < MINVAL) { a[0] = 1; a[1] = a[2] = 0; return n; }
  a[0] /= n; a[1] /= n; a[2] /= n;
  return n;
}
static void axis_angle_quat(double q[4], const double ax[3], double ang) {
  double s = sin(ang / 2);
  q[0] = cos(ang / 2); q[1] = ax[0] * s; q[2] = ax[1] * s; q[3] = ax[2] * s;
}
static void mat_mul(double r[9], const double a[9], const double b[9]) {
  double t[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) t[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
  memcpy(r, t, sizeof t);
}
/* spatial algebra [upstream engine_util_spatial.c]: motion/force vectors are (angular, linear) */
static void mul_inert_vec(double r[6], const double i[10], const double v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
static void cross_motion(double r[6], const double v[6], const double u[6]) {
  double t[6];
  t[0] = -v[2] * u[1] + v[1] * u[2];
  t[1] = v[2] * u[0] - v[0] * u[2];
  t[2] = -v[1] * u[0] + v[0] * u[1];
  t[3] = -v[2] * u[4] + v[1] * u[5] - v[5] * u[1] + v[4] * u[2];
  t[4] = v[2] * u[3] - v[0] * u[5] + v[5] * u[0] - v[3] * u[2];
  t[5] = -v[1] * u[3] + v[0] * u[4] - v[4] * u[0] + v[3] * u[1];
  memcpy(r, t, sizeof t);
}
static void cross_force(double r[6], const double v[6], const double f[6]) {
  double t[6];
  t[0] = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  t[1] = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  t[2] = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  t[3] = -v[2] * f[4] + v[1] * f[5];
  t[4] = v[2] * f[3] - v[0] * f[5];
  t[5] = -v[1] * f[3] + v[0] * f[4];
  memcpy(r, t, sizeof t);
}
static int is_bad(double x) { return isnan(x) || x > MAXVAL || x < -MAXVAL; }

/* ------------------------------------------------------------------------ data */
static double* dalloc(size_t n) { return (double*)calloc(n ? n : 1, sizeof(double)); }

orc_data* orc_make_data(const mrs_model_view* m) {
  orc_data* d = (orc_data*)calloc(1, sizeof(orc_data));
  d->qpos = dalloc(m->nq); d->qvel = dalloc(m->nv); d->ctrl = dalloc(m->nu);
  d->qfrc_applied = dalloc(m->nv); d->qacc_warmstart = dalloc(m->nv); d->qacc = dalloc(m->nv);
  d->qfrc_actuator = dalloc(m->nv); d->sensordata = dalloc(m->nsensordata);
  orc_ws* w = (orc_ws*)calloc(1, sizeof(orc_ws));
  int nb = m->nbody, nv = m->nv, nj = m->njnt, ng = m->ngeom;
  w->xpos = dalloc(3 * nb); w->xquat = dalloc(4 * nb); w->xmat = dalloc(9 * nb);
  w->xipos = dalloc(3 * nb); w->ximat = dalloc(9 * nb); w->xanchor = dalloc(3 * nj);
  w->xaxis = dalloc(3 * nj); w->geom_xpos = dalloc(3 * ng); w->geom_xmat = dalloc(9 * ng);
  w->subtree_com = dalloc(3 * nb); w->cinert = dalloc(10 * nb); w->cdof = dalloc(6 * nv);
  w->crb = dalloc(10 * nb); w->cvel = dalloc(6 * nb); w->cdof_dot = dalloc(6 * nv);
  w->cacc = dalloc(6 * nb); w->cfrc = dalloc(6 * nb);
  w->cacc_full = dalloc(6 * nb); w->cfrc_ext = dalloc(6 * nb); w->cfrc_int = dalloc(6 * nb);
  w->M = dalloc(nv * nv); w->L = dalloc(nv * nv); w->Mi = dalloc(nv * nv); w->Li = dalloc(nv * nv);
  w->qfrc_bias = dalloc(nv); w->qfrc_passive = dalloc(nv); w->qfrc_smooth = dalloc(nv);
  w->qacc_smooth = dalloc(nv); w->qfrc_constraint = dalloc(nv); w->actuator_force = dalloc(m->nu);
  w->tmp = dalloc(nv > 6 ? nv : 6); w->tmp2 = dalloc(nv > 6 ? nv : 6);
  w->efc_J = dalloc((size_t)MAXEFC * nv); w->efc_MinvJT = dalloc((size_t)MAXEFC * nv);
  w->AR = NULL;
  d->ws = w;
  orc_reset(m, d, -1);
  return d;
}

void orc_free_data(orc_data* d) {
  if (!d) return;
  orc_ws* w = (orc_ws*)d->ws;
  double* arrs[] = {w->xpos, w->xquat, w->xmat, w->xipos, w->ximat, w->xanchor, w->xaxis,
                    w->geom_xpos, w->geom_xmat, w->subtree_com, w->cinert, w->cdof, w->crb,
                    w->cvel, w->cdof_dot, w->cacc, w->cfrc, w->M, w->L, w->Mi, w->Li,
                    w->qfrc_bias, w->qfrc_passive, w->qfrc_smooth, w->qacc_smooth,
                    w->qfrc_constraint, w->actuator_force, w->tmp, w->tmp2, w->efc_J,
                    w->efc_MinvJT, w->AR, w->cacc_full, w->cfrc_ext, w->cfrc_int};
  for (size_t i = 0; i < sizeof arrs / sizeof arrs[0]; ++i) free(arrs[i]);
  free(w);
  free(d->qpos); free(d->qvel); free(d->ctrl); free(d->qfrc_applied); free(d->qacc_warmstart);
  free(d->qacc); free(d->qfrc_actuator); free(d->sensordata);
  free(d);
}

/* mj_resetData / mj_resetDataKeyframe [upstream engine_io.c] */
void orc_reset(const mrs_model_view* m, orc_data* d, int key) {
  if (m->nq > 0) memcpy(d->qpos, m->qpos0, sizeof(double) * m->nq);  /* (an empty model has no arrays) */
  memset(d->qvel, 0, sizeof(double) * m->nv);
  memset(d->ctrl, 0, sizeof(double) * m->nu);
  memset(d->qfrc_applied, 0, sizeof(double) * m->nv);
  memset(d->qacc_warmstart, 0, sizeof(double) * m->nv);
  memset(d->qacc, 0, sizeof(double) * m->nv);
  memset(d->qfrc_actuator, 0, sizeof(double) * m->nv);
  memset(d->sensordata, 0, sizeof(double) * m->nsensordata);
  d->time = 0;
  if (key >= 0 && key < m->nkey) {
    d->time = m->key_time[key];
    if (m->nq > 0) memcpy(d->qpos, m->key_qpos + (size_t)key * m->nq, sizeof(double) * m->nq);
    if (m->nv > 0) memcpy(d->qvel, m->key_qvel + (size_t)key * m->nv, sizeof(double) * m->nv);
    if (m->nu > 0) memcpy(d->ctrl, m->key_ctrl + (size_t)key * m->nu, sizeof(double) * m->nu);
  }
}

/* ------------------------------------------------------------------------ kinematics
 * mj_kinematics [upstream engine_core_smooth.c]: body frames from parent, joints applied in order
 * (hinge: rotate about axis through anchor by qpos-qpos0; slide: translate; ball: quaternion;
 * free: world pose from qpos), then inertial frames and geom frames. */
static void kinematics(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  w->xpos[0] = w->xpos[1] = w->xpos[2] = 0;
  w->xquat[0] = 1; w->xquat[1] = w->xquat[2] = w->xquat[3] = 0;
  quat2mat(w->xmat, w->xquat);
  memcpy(w->ximat, w->xmat, 9 * sizeof(double));
  memset(w->xipos, 0, 3 * sizeof(double));
  for (int b = 1; b < m->nbody; ++b) {
    int p = m->body_parentid[b];
    double* pos = w->xpos + 3 * b;
    double* q = w->xquat + 4 * b;
    int ja = m->body_jntadr[b];
    if (m->body_jntnum[b] > 0 && m->jnt_type[ja] == MRS_JNT_FREE) {
      const double* qp = d->qpos + m->jnt_qposadr[ja];
      pos[0] = qp[0]; pos[1] = qp[1]; pos[2] = qp[2];
      q[0] = qp[3]; q[1] = qp[4]; q[2] = qp[5]; q[3] = qp[6];
      quat_normalize(q);
      memcpy(w->xanchor + 3 * ja, pos, 3 * sizeof(double));
      memset(w->xaxis + 3 * ja, 0, 3 * sizeof(double));
    } else {
      double r[3];
      rot_quat(r, m->body_pos + 3 * b, w->xquat + 4 * p);
      for (int i = 0; i < 3; ++i) pos[i] = w->xpos[3 * p + i] + r[i];
      quat_mul(q, w->xquat + 4 * p, m->body_quat + 4 * b);
      for (int k = 0; k < m->body_jntnum[b]; ++k) {
        int j = ja + k, a = m->jnt_qposadr[j];
        double* anc = w->xanchor + 3 * j;
        double* ax = w->xaxis + 3 * j;
        rot_quat(anc, m->jnt_pos + 3 * j, q);
        for (int i = 0; i < 3; ++i) anc[i] += pos[i];
        rot_quat(ax, m->jnt_axis + 3 * j, q);
        if (m->jnt_type[j] == MRS_JNT_SLIDE) {
          double dq = d->qpos[a] - m->qpos0[a];
          for (int i = 0; i < 3; ++i) pos[i] += ax[i] * dq;
        } else {
          double qloc[4];
          if (m->jnt_type[j] == MRS_JNT_BALL) {
            memcpy(qloc, d->qpos + a, 4 * sizeof(double));
            quat_normalize(qloc);
          } else {
            axis_angle_quat(qloc, m->jnt_axis + 3 * j, d->qpos[a] - m->qpos0[a]);
          }
          quat_mul(q, q, qloc);
          double v[3];
          rot_quat(v, m->jnt_pos + 3 * j, q);
          for (int i = 0; i < 3; ++i) pos[i] = anc[i] - v[i];
        }
      }
    }
    quat_normalize(q);
    quat2mat(w->xmat + 9 * b, q);
    double r[3], iq[4];
    rot_quat(r, m->body_ipos + 3 * b, q);
    for (int i = 0; i < 3; ++i) w->xipos[3 * b + i] = pos[i] + r[i];
    quat_mul(iq, q, m->body_iquat + 4 * b);
    quat2mat(w->ximat + 9 * b, iq);
  }
  for (int g = 0; g < m->ngeom; ++g) {
    int b = m->geom_bodyid[g];
    double r[3], gq[4];
    rot_quat(r, m->geom_pos + 3 * g, w->xquat + 4 * b);
    for (int i = 0; i < 3; ++i) w->geom_xpos[3 * g + i] = w->xpos[3 * b + i] + r[i];
    quat_mul(gq, w->xquat + 4 * b, m->geom_quat + 4 * g);
    quat2mat(w->geom_xmat + 9 * g, gq);
  }
}

/* site world pose (mj_kinematics site loop) */
static void site_pose(const mrs_model_view* m, orc_ws* w, int s, double pos[3], double mat[9]) {
  int b = m->site_bodyid[s];
  double r[3], q[4];
  rot_quat(r, m->site_pos + 3 * s, w->xquat + 4 * b);
  for (int i = 0; i < 3; ++i) pos[i] = w->xpos[3 * b + i] + r[i];
  quat_mul(q, w->xquat + 4 * b, m->site_quat + 4 * s);
  quat2mat(mat, q);
}

/* mj_comPos [upstream]: subtree centres of mass, com-based inertias (cinert), motion dofs (cdof) */
static void com_pos(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  int nb = m->nbody;
  for (int b = 0; b < nb; ++b)
    for (int i = 0; i < 3; ++i) w->subtree_com[3 * b + i] = m->body_mass[b] * w->xipos[3 * b + i];
  for (int b = nb - 1; b > 0; --b)
    for (int i = 0; i < 3; ++i) w->subtree_com[3 * m->body_parentid[b] + i] += w->subtree_com[3 * b + i];
  for (int b = 0; b < nb; ++b)
    for (int i = 0; i < 3; ++i)
      w->subtree_com[3 * b + i] = m->body_subtreemass[b] > MINVAL
                                      ? w->subtree_com[3 * b + i] / m->body_subtreemass[b]
                                      : w->xipos[3 * b + i];
  memset(w->cinert, 0, 10 * sizeof(double));
  for (int b = 1; b < nb; ++b) {
    const double* mat = w->ximat + 9 * b;
    const double* in = m->body_inertia + 3 * b;
    double mass = m->body_mass[b], dif[3], full[9];
    for (int i = 0; i < 3; ++i) dif[i] = w->xipos[3 * b + i] - w->subtree_com[3 * m->body_rootid[b] + i];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        full[3 * r + c] = mat[3 * r] * in[0] * mat[3 * c] + mat[3 * r + 1] * in[1] * mat[3 * c + 1] +
                          mat[3 * r + 2] * in[2] * mat[3 * c + 2];
    double* ci = w->cinert + 10 * b;
    ci[0] = full[0] + mass * (dif[1] * dif[1] + dif[2] * dif[2]);
    ci[1] = full[4] + mass * (dif[0] * dif[0] + dif[2] * dif[2]);
    ci[2] = full[8] + mass * (dif[0] * dif[0] + dif[1] * dif[1]);
    ci[3] = full[1] - mass * dif[0] * dif[1];
    ci[4] = full[2] - mass * dif[0] * dif[2];
    ci[5] = full[5] - mass * dif[1] * dif[2];
    ci[6] = mass * dif[0]; ci[7] = mass * dif[1]; ci[8] = mass * dif[2]; ci[9] = mass;
  }
  for (int j = 0; j < m->njnt; ++j) {
    int b = m->jnt_bodyid[j], dof = m->jnt_dofadr[j];
    const double* c = w->subtree_com + 3 * m->body_rootid[b];
    double off[3];
    for (int i = 0; i < 3; ++i) off[i] = c[i] - w->xanchor[3 * j + i];
    double* cd;
    switch (m->jnt_type[j]) {
      case MRS_JNT_HINGE:
        cd = w->cdof + 6 * dof;
        memcpy(cd, w->xaxis + 3 * j, 3 * sizeof(double));
        cross3(cd + 3, cd, off);
        break;
      case MRS_JNT_SLIDE:
        cd = w->cdof + 6 * dof;
        cd[0] = cd[1] = cd[2] = 0;
        memcpy(cd + 3, w->xaxis + 3 * j, 3 * sizeof(double));
        break;
      case MRS_JNT_FREE:
        for (int k = 0; k < 3; ++k) {
          cd = w->cdof + 6 * (dof + k);
          for (int i = 0; i < 6; ++i) cd[i] = (i == 3 + k) ? 1 : 0;
        }
        dof += 3;
        /* fall through */
      case MRS_JNT_BALL:
        for (int k = 0; k < 3; ++k) {
          cd = w->cdof + 6 * (dof + k);
          const double* xm = w->xmat + 9 * b;
          cd[0] = xm[k]; cd[1] = xm[3 + k]; cd[2] = xm[6 + k];
          cross3(cd + 3, cd, off);
        }
        break;
    }
  }
}

/* mj_crb + armature [upstream mj_makeM]: composite inertias, dense symmetric M */
static void make_M(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  int nb = m->nbody, nv = m->nv;
  memcpy(w->crb, w->cinert, 10 * nb * sizeof(double));
  for (int b = nb - 1; b > 0; --b)
    if (m->body_parentid[b] > 0)
      for (int i = 0; i < 10; ++i) w->crb[10 * m->body_parentid[b] + i] += w->crb[10 * b + i];
  memset(w->M, 0, (size_t)nv * nv * sizeof(double));
  for (int i = 0; i < nv; ++i) {
    double buf[6];
    mul_inert_vec(buf, w->crb + 10 * m->dof_bodyid[i], w->cdof + 6 * i);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      double v = 0;
      for (int k = 0; k < 6; ++k) v += w->cdof[6 * j + k] * buf[k];
      w->M[i * nv + j] = w->M[j * nv + i] = v;
    }
    w->M[i * nv + i] += m->dof_armature[i];
  }
}

/* dense Cholesky A = L L' (lower).  MuJoCo factors M as sparse L'DL (mj_factorM); the factor
 * differs but the solves are mathematically identical. */
static void cholesky(const double* A, double* L, int n) {
  memset(L, 0, (size_t)n * n * sizeof(double));
  for (int j = 0; j < n; ++j) {
    double s = A[j * n + j];
    for (int k = 0; k < j; ++k) s -= L[j * n + k] * L[j * n + k];
    L[j * n + j] = sqrt(s > MINVAL ? s : MINVAL);
    for (int i = j + 1; i < n; ++i) {
      double t = A[i * n + j];
      for (int k = 0; k < j; ++k) t -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = t / L[j * n + j];
    }
  }
}
static void chol_solve(const double* L, double* x, const double* b, int n) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int k = 0; k < i; ++k) s -= L[i * n + k] * x[k];
    x[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = x[i];
    for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * x[k];
    x[i] = s / L[i * n + i];
  }
}

/* mj_comVel [upstream]: body spatial velocities and cdof_dot = cvel x cdof (parent velocity) */
static void com_vel(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  memset(w->cvel, 0, 6 * sizeof(double));
  for (int b = 1; b < m->nbody; ++b) {
    double cv[6];
    memcpy(cv, w->cvel + 6 * m->body_parentid[b], sizeof cv);
    int da = m->body_dofadr[b];
    for (int k = 0; k < m->body_dofnum[b]; ++k) {
      int j = da + k;
      int jt = m->jnt_type[m->dof_jntid[j]];
      if (jt == MRS_JNT_FREE && j == m->jnt_dofadr[m->dof_jntid[j]]) {
        for (int t = 0; t < 3; ++t) {
          memset(w->cdof_dot + 6 * (j + t), 0, 6 * sizeof(double));
          for (int i = 0; i < 6; ++i) cv[i] += w->cdof[6 * (j + t) + i] * d->qvel[j + t];
        }
        k += 2;
        continue;
      }
      if (jt == MRS_JNT_BALL || jt == MRS_JNT_FREE) {
        /* rotational triple: cdof_dot with the velocity before the triple is added */
        for (int t = 0; t < 3; ++t) cross_motion(w->cdof_dot + 6 * (j + t), cv, w->cdof + 6 * (j + t));
        for (int t = 0; t < 3; ++t)
          for (int i = 0; i < 6; ++i) cv[i] += w->cdof[6 * (j + t) + i] * d->qvel[j + t];
        k += 2;
        continue;
      }
      cross_motion(w->cdof_dot + 6 * j, cv, w->cdof + 6 * j);
      for (int i = 0; i < 6; ++i) cv[i] += w->cdof[6 * j + i] * d->qvel[j];
    }
    memcpy(w->cvel + 6 * b, cv, sizeof cv);
  }
}

/* mj_rne with flg_acc = 0 [upstream]: qfrc_bias = C(q,v) + g(q) */
static void rne(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  int nb = m->nbody;
  memset(w->cacc, 0, 6 * sizeof(double));
  if (!(m->disableflags & MRS_DSBL_GRAVITY))
    for (int i = 0; i < 3; ++i) w->cacc[3 + i] = -m->gravity[i];
  memset(w->cfrc, 0, 6 * sizeof(double));
  for (int b = 1; b < nb; ++b) {
    double* ca = w->cacc + 6 * b;
    memcpy(ca, w->cacc + 6 * m->body_parentid[b], 6 * sizeof(double));
    int da = m->body_dofadr[b];
    for (int k = 0; k < m->body_dofnum[b]; ++k)
      for (int i = 0; i < 6; ++i) ca[i] += w->cdof_dot[6 * (da + k) + i] * d->qvel[da + k];
    double f1[6], t[6], f2[6];
    mul_inert_vec(f1, w->cinert + 10 * b, ca);
    mul_inert_vec(t, w->cinert + 10 * b, w->cvel + 6 * b);
    cross_force(f2, w->cvel + 6 * b, t);
    for (int i = 0; i < 6; ++i) w->cfrc[6 * b + i] = f1[i] + f2[i];
  }
  for (int b = nb - 1; b > 0; --b)
    if (m->body_parentid[b] > 0)
      for (int i = 0; i < 6; ++i) w->cfrc[6 * m->body_parentid[b] + i] += w->cfrc[6 * b + i];
  for (int j = 0; j < m->nv; ++j) {
    double v = 0;
    for (int i = 0; i < 6; ++i) v += w->cdof[6 * j + i] * w->cfrc[6 * m->dof_bodyid[j] + i];
    w->qfrc_bias[j] = v;
  }
}

/* does dof j move body b (j in b's dof chain)? */
static int dof_affects(const mrs_model_view* m, int j, int b) {
  int bj = m->dof_bodyid[j];
  for (int x = b; x != 0; x = m->body_parentid[x])
    if (x == bj) return 1;
  return 0;
}

/* mj_jac translational part [upstream engine_core_smooth.c]: column j of the point Jacobian of a
 * point attached to body b */
static void jac_point_col(const mrs_model_view* m, orc_ws* w, int b, const double pnt[3], int j,
                          double col[3]) {
  double off[3], cr[3];
  for (int i = 0; i < 3; ++i) off[i] = pnt[i] - w->subtree_com[3 * m->body_rootid[b] + i];
  cross3(cr, w->cdof + 6 * j, off);
  for (int i = 0; i < 3; ++i) col[i] = w->cdof[6 * j + 3 + i] + cr[i];
}

/* fixed tendon t [upstream mj_tendon, fixed tendons]: length sum_k coef_k qpos_k; velocity and the
 * constant Jacobian row J (nv, may be NULL) from the wrapped joints' dofs */
static double tendon_length(const mrs_model_view* m, const orc_data* d, int t, double* J, double* vel) {
  double L = 0, v = 0;
  if (J) memset(J, 0, m->nv * sizeof(double));
  for (int k = m->tendon_adr[t]; k < m->tendon_adr[t] + m->tendon_num[t]; ++k) {
    const int j = m->wrap_objid[k];
    const double c = m->wrap_prm[k];
    L += c * d->qpos[m->jnt_qposadr[j]];
    v += c * d->qvel[m->jnt_dofadr[j]];
    if (J) J[m->jnt_dofadr[j]] += c;
  }
  if (vel) *vel = v;
  return L;
}

/* mj_passive [upstream engine_passive.c]: joint springs, dampers, tendon springs (dead band
 * [lengthspring0, lengthspring1]) and dampers through J', gravity compensation */
static void passive(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  memset(w->qfrc_passive, 0, m->nv * sizeof(double));
  if (m->disableflags & MRS_DSBL_PASSIVE) return;
  for (int j = 0; j < m->njnt; ++j) {
    int t = m->jnt_type[j];
    if ((t == MRS_JNT_HINGE || t == MRS_JNT_SLIDE) && m->jnt_stiffness[j] != 0) {
      int a = m->jnt_qposadr[j];
      w->qfrc_passive[m->jnt_dofadr[j]] -= m->jnt_stiffness[j] * (d->qpos[a] - m->qpos_spring[a]);
    }
  }
  for (int i = 0; i < m->nv; ++i) w->qfrc_passive[i] -= m->dof_damping[i] * d->qvel[i];
  if (m->ntendon > 0) {
    double* J = (double*)malloc(m->nv * sizeof(double) + 8);
    for (int t = 0; t < m->ntendon; ++t) {
      const double k = m->tendon_stiffness[t], b = m->tendon_damping[t];
      if (k == 0 && b == 0) continue;
      double v;
      const double L = tendon_length(m, d, t, J, &v);
      const double* ls = m->tendon_lengthspring + 2 * t;
      double f = 0;
      if (k != 0) f = L > ls[1] ? k * (ls[1] - L) : (L < ls[0] ? k * (ls[0] - L) : 0);
      f -= b * v;
      for (int i = 0; i < m->nv; ++i) w->qfrc_passive[i] += J[i] * f;
    }
    free(J);
  }
  if (!(m->disableflags & MRS_DSBL_GRAVITY)) {
    for (int b = 1; b < m->nbody; ++b) {
      if (m->body_gravcomp[b] == 0) continue;
      double f[3];
      for (int i = 0; i < 3; ++i) f[i] = -m->gravity[i] * m->body_mass[b] * m->body_gravcomp[b];
      for (int j = 0; j < m->nv; ++j) {
        if (!dof_affects(m, j, b)) continue;
        double col[3];
        jac_point_col(m, w, b, w->xipos + 3 * b, j, col);
        w->qfrc_passive[j] += dot3(col, f);
      }
    }
  }
}

/* mj_fwdActuation [upstream engine_forward.c] for joint transmissions without dynamics */
static void actuation(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  memset(d->qfrc_actuator, 0, m->nv * sizeof(double));
  if (m->disableflags & MRS_DSBL_ACTUATION) { memset(w->actuator_force, 0, m->nu * sizeof(double)); return; }
  double* Jt = m->ntendon > 0 ? (double*)malloc(m->nv * sizeof(double) + 8) : NULL;
  for (int a = 0; a < m->nu; ++a) {
    int j = m->actuator_trnid[2 * a];
    const int tendon = m->actuator_trntype[a] == MRS_TRN_TENDON;
    int qa = tendon ? 0 : m->jnt_qposadr[j], da = tendon ? 0 : m->jnt_dofadr[j];
    double gear = m->actuator_gear[6 * a];
    double len, vel;
    if (tendon) {
      double tv;
      len = gear * tendon_length(m, d, j, Jt, &tv);
      vel = gear * tv;
    } else {
      len = gear * d->qpos[qa];
      vel = gear * d->qvel[da];
    }
    double ctrl = d->ctrl[a];
    if (m->actuator_ctrllimited[a] && !(m->disableflags & MRS_DSBL_CLAMPCTRL)) {
      const double* r = m->actuator_ctrlrange + 2 * a;
      ctrl = ctrl < r[0] ? r[0] : ctrl > r[1] ? r[1] : ctrl;
    }
    const double* g = m->actuator_gainprm + MRS_NGAIN * a;
    const double* bp = m->actuator_biasprm + MRS_NBIAS * a;
    double gain = g[0];
    if (m->actuator_gaintype[a] == MRS_GAIN_AFFINE) gain = g[0] + g[1] * len + g[2] * vel;
    double bias = 0;
    if (m->actuator_biastype[a] == MRS_BIAS_AFFINE) bias = bp[0] + bp[1] * len + bp[2] * vel;
    double force = gain * ctrl + bias;
    if (m->actuator_forcelimited[a]) {
      const double* r = m->actuator_forcerange + 2 * a;
      force = force < r[0] ? r[0] : force > r[1] ? r[1] : force;
    }
    w->actuator_force[a] = force;
    if (tendon)
      for (int i = 0; i < m->nv; ++i) d->qfrc_actuator[i] += gear * force * Jt[i];
    else
      d->qfrc_actuator[da] += gear * force;
  }
  free(Jt);
  for (int j = 0; j < m->njnt; ++j) {
    if (!m->jnt_actfrclimited[j]) continue;
    const double* r = m->jnt_actfrcrange + 2 * j;
    int da = m->jnt_dofadr[j];
    int n = m->jnt_type[j] == MRS_JNT_FREE ? 6 : m->jnt_type[j] == MRS_JNT_BALL ? 3 : 1;
    for (int k = 0; k < n; ++k) {
      double v = d->qfrc_actuator[da + k];
      d->qfrc_actuator[da + k] = v < r[0] ? r[0] : v > r[1] ? r[1] : v;
    }
  }
}

/* ------------------------------------------------------------------------ collision
 * Broad phase: every geom pair (g1 < g2) passing MuJoCo's filters [upstream engine_collision_driver.c
 * mj_collision/filterBodyPair]: distinct weld bodies, not both static, parent-child weld filter,
 * contype/conaffinity, bounding-sphere distance with margin.  Narrow phase: analytic primitives
 * (plane-sphere/capsule/box, sphere-sphere, sphere-capsule, capsule-capsule, sphere-box,
 * capsule-box).  Contact order = pair order, then the primitive's own order. */
static void make_frame(double f[9]) {
  normalize3(f);
  if (fabs(f[1]) < 0.5) { f[3] = 0; f[4] = 1; f[5] = 0; }
  else { f[3] = 0; f[4] = 0; f[5] = 1; }
  double dd = dot3(f, f + 3);
  for (int i = 0; i < 3; ++i) f[3 + i] -= dd * f[i];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}
static int add_contact(orc_contact* out, int n, double dist, const double pos[3], const double nrm[3]) {
  if (n >= 8) return n; /* a pair gives at most 8 contacts (box-box face polygon) */
  orc_contact* c = out + n;
  c->dist = dist;
  memcpy(c->pos, pos, 3 * sizeof(double));
  memcpy(c->frame, nrm, 3 * sizeof(double));
  make_frame(c->frame);
  return n + 1;
}
static int col_sphere_sphere(const double p1[3], double r1, const double p2[3], double r2,
                             double margin, orc_contact* out, int n) {
  double dv[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double len = norm3(dv);
  double dist = len - r1 - r2;
  if (dist > margin) return n;
  double nrm[3];
  if (len < MINVAL) { nrm[0] = 1; nrm[1] = nrm[2] = 0; }
  else { nrm[0] = dv[0] / len; nrm[1] = dv[1] / len; nrm[2] = dv[2] / len; }
  double pos[3];
  for (int i = 0; i < 3; ++i) pos[i] = p1[i] + nrm[i] * (r1 + dist / 2);
  return add_contact(out, n, dist, pos, nrm);
}
static void segment_point_closest(const double a[3], const double b[3], const double p[3], double c[3]) {
  double ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
  double den = dot3(ab, ab), t = den > MINVAL ? dot3(ap, ab) / den : 0;
  t = t < 0 ? 0 : t > 1 ? 1 : t;
  for (int i = 0; i < 3; ++i) c[i] = a[i] + t * ab[i];
}
/* closest points of two segments (clamped parametric form) */
static void segment_segment_closest(const double a0[3], const double a1[3], const double b0[3],
                                    const double b1[3], double ca[3], double cb[3]) {
  double d1[3] = {a1[0] - a0[0], a1[1] - a0[1], a1[2] - a0[2]};
  double d2[3] = {b1[0] - b0[0], b1[1] - b0[1], b1[2] - b0[2]};
  double r[3] = {a0[0] - b0[0], a0[1] - b0[1], a0[2] - b0[2]};
  double a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  double s = 0, t = 0;
  if (a <= MINVAL && e <= MINVAL) { s = t = 0; }
  else if (a <= MINVAL) { s = 0; t = f / e; t = t < 0 ? 0 : t > 1 ? 1 : t; }
  else {
    double c = dot3(d1, r);
    if (e <= MINVAL) { t = 0; s = -c / a; s = s < 0 ? 0 : s > 1 ? 1 : s; }
    else {
      double bb = dot3(d1, d2), den = a * e - bb * bb;
      s = den > MINVAL * a * e ? (bb * f - c * e) / den : 0;
      s = s < 0 ? 0 : s > 1 ? 1 : s;
      t = (bb * s + f) / e;
      if (t < 0) { t = 0; s = -c / a; s = s < 0 ? 0 : s > 1 ? 1 : s; }
      else if (t > 1) { t = 1; s = (bb - c) / a; s = s < 0 ? 0 : s > 1 ? 1 : s; }
    }
  }
  for (int i = 0; i < 3; ++i) { ca[i] = a0[i] + s * d1[i]; cb[i] = b0[i] + t * d2[i]; }
}
static void capsule_ends(const double* pos, const double* mat, double hl, double a[3], double b[3]) {
  for (int i = 0; i < 3; ++i) { a[i] = pos[i] - mat[3 * i + 2] * hl; b[i] = pos[i] + mat[3 * i + 2] * hl; }
}
/* plane (geom1) vs sphere at p with radius r */
static int col_plane_sphere(const double* ppos, const double* pmat, const double p[3], double r,
                            double margin, orc_contact* out, int n) {
  double nrm[3] = {pmat[2], pmat[5], pmat[8]};
  double dv[3] = {p[0] - ppos[0], p[1] - ppos[1], p[2] - ppos[2]};
  double dist = dot3(dv, nrm) - r;
  if (dist > margin) return n;
  double pos[3];
  for (int i = 0; i < 3; ++i) pos[i] = p[i] - nrm[i] * (r + dist / 2);
  return add_contact(out, n, dist, pos, nrm);
}
static int col_plane_box(const double* ppos, const double* pmat, const double* bpos, const double* bmat,
                         const double* size, double margin, orc_contact* out, int n) {
  double nrm[3] = {pmat[2], pmat[5], pmat[8]};
  double dv[3] = {bpos[0] - ppos[0], bpos[1] - ppos[1], bpos[2] - ppos[2]};
  double cdist = dot3(dv, nrm);
  for (int k = 0; k < 8 && n < 4; ++k) {
    double v[3] = {(k & 1) ? size[0] : -size[0], (k & 2) ? size[1] : -size[1], (k & 4) ? size[2] : -size[2]};
    double c[3];
    mat_vec(c, bmat, v);
    double ld = dot3(nrm, c);
    double dist = cdist + ld;
    if (dist > margin || ld > 0) continue;
    double pos[3];
    for (int i = 0; i < 3; ++i) pos[i] = bpos[i] + c[i] - nrm[i] * dist / 2;
    n = add_contact(out, n, dist, pos, nrm);
  }
  return n;
}
/* sphere (center p, radius r) vs box (geom2): normal points from sphere to box */
static int col_sphere_box(const double p[3], double r, const double* bpos, const double* bmat,
                          const double* size, double margin, orc_contact* out, int n) {
  double dv[3] = {p[0] - bpos[0], p[1] - bpos[1], p[2] - bpos[2]}, l[3];
  matT_vec(l, bmat, dv);
  double c[3];
  int inside = 1;
  for (int i = 0; i < 3; ++i) {
    c[i] = l[i] < -size[i] ? -size[i] : l[i] > size[i] ? size[i] : l[i];
    if (c[i] != l[i]) inside = 0;
  }
  double nrm_l[3], dist;
  if (!inside) {
    double dl[3] = {c[0] - l[0], c[1] - l[1], c[2] - l[2]};
    double len = norm3(dl);
    dist = len - r;
    if (dist > margin) return n;
    for (int i = 0; i < 3; ++i) nrm_l[i] = dl[i] / len;
  } else {
    /* centre inside: push out through the nearest face */
    int ax = 0;
    double best = 1e300;
    for (int i = 0; i < 3; ++i) {
      double pen = size[i] - fabs(l[i]);
      if (pen < best) { best = pen; ax = i; }
    }
    dist = -best - r;
    nrm_l[0] = nrm_l[1] = nrm_l[2] = 0;
    nrm_l[ax] = l[ax] >= 0 ? -1 : 1;
    c[ax] = l[ax] >= 0 ? size[ax] : -size[ax];
  }
  double nrm[3], pos[3];
  mat_vec(nrm, bmat, nrm_l);
  /* contact point halfway between the sphere surface and the box surface */
  for (int i = 0; i < 3; ++i) pos[i] = p[i] + nrm[i] * (r + dist / 2);
  return add_contact(out, n, dist, pos, nrm);
}
/* capsule (segment a-b, radius r) vs box.  In the box frame the squared distance of the segment
 * point at t to the box, F(t) = sum_i max(0, |la_i + t d_i| - s_i)^2, is convex and piecewise
 * quadratic with breakpoints where a coordinate crosses a slab plane (la_i + t d_i = +-s_i): the exact
 * minimiser t* is the best of the pieces' clamped stationary points.  Contacts (restated primitive,
 * well conditioned in fp32 and fp64 alike):
 *   - the segment is clipped to the slabs |l_j| <= s_j of the axes on which the closest point t* lies
 *     inside the box's extent (the face or edge it is closest to);
 *   - when t* lies strictly inside that piece and is clearly nearer than both its ends (a capsule
 *     across an edge), by more than 1e-6 + 1e-4 r, the closest point alone is the contact;
 *   - otherwise the two ends of the piece, where within margin, are the contacts -- a capsule lying on
 *     a face rests on two points whatever its overhang, where the single closest point would be
 *     arbitrary along the face;
 *   - a segment that passes through the box (F(t*) = 0): the point of deepest penetration, found by
 *     ternary search on the concave min_i (s_i - |l_i(t)|).
 * At most 2 contacts, as MuJoCo's mjc_CapsuleBox (the closest point, plus a second one for a capsule
 * parallel to a face); which points its selection takes in the flat case is not restated [verify].
 * Same algorithm as step.hip capsule_box. */
static double seg_box_F(const double la[3], const double d[3], const double* s, double t) {
  double f = 0;
  for (int i = 0; i < 3; ++i) {
    double e = fabs(la[i] + t * d[i]) - s[i];
    if (e > 0) f += e * e;
  }
  return f;
}
static double seg_box_closest(const double la[3], const double d[3], const double* s, double* Fbest) {
  double bp[8];
  bp[0] = 0;
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 2; ++k) {
      double t = 1;
      if (fabs(d[i]) > 1e-12) {
        t = ((k ? s[i] : -s[i]) - la[i]) / d[i];
        if (!(t > 0 && t < 1)) t = 1;
      }
      bp[1 + 2 * i + k] = t;
    }
  bp[7] = 1;
  for (int i = 1; i < 8; ++i)  /* insertion sort */
    for (int j = i; j > 0 && bp[j] < bp[j - 1]; --j) { double x = bp[j]; bp[j] = bp[j - 1]; bp[j - 1] = x; }
  double best_t = 0, best_F = seg_box_F(la, d, s, 0);
  for (int k = 0; k < 7; ++k) {
    double t0 = bp[k], t1 = bp[k + 1];
    if (!(t1 > t0)) continue;
    double tm = 0.5 * (t0 + t1), num = 0, den = 0;
    for (int i = 0; i < 3; ++i) {
      double x = la[i] + tm * d[i];
      if (fabs(x) > s[i]) {
        double sg = x > 0 ? 1 : -1;
        num += d[i] * (la[i] - sg * s[i]);
        den += d[i] * d[i];
      }
    }
    double t = den > 0 ? -num / den : t0;
    t = t < t0 ? t0 : t > t1 ? t1 : t;
    double F = seg_box_F(la, d, s, t);
    if (F < best_F) { best_F = F; best_t = t; }
  }
  *Fbest = best_F;
  return best_t;
}
static int col_capsule_box(const double a[3], const double b[3], double r, const double* bpos,
                           const double* bmat, const double* size, double margin, orc_contact* out, int n) {
  double da[3] = {a[0] - bpos[0], a[1] - bpos[1], a[2] - bpos[2]}, db[3], la[3], lb[3], d[3];
  for (int i = 0; i < 3; ++i) db[i] = b[i] - bpos[i];
  matT_vec(la, bmat, da);
  matT_vec(lb, bmat, db);
  for (int i = 0; i < 3; ++i) d[i] = lb[i] - la[i];
  double Fbest;
  double t = seg_box_closest(la, d, size, &Fbest);
  double p[3];
  if (Fbest <= 0) {
    /* the segment passes through the box: deepest point of min_i (s_i - |l_i(t)|) */
    double lo = 0, hi = 1;
    for (int it = 0; it < 40; ++it) {
      double t1 = lo + (hi - lo) / 3, t2 = hi - (hi - lo) / 3, p1 = 1e300, p2 = 1e300;
      for (int i = 0; i < 3; ++i) {
        double e1 = size[i] - fabs(la[i] + t1 * d[i]), e2 = size[i] - fabs(la[i] + t2 * d[i]);
        p1 = e1 < p1 ? e1 : p1;
        p2 = e2 < p2 ? e2 : p2;
      }
      if (p1 >= p2) hi = t2;
      else lo = t1;
    }
    t = 0.5 * (lo + hi);
    for (int i = 0; i < 3; ++i) p[i] = a[i] + t * (b[i] - a[i]);
    return col_sphere_box(p, r, bpos, bmat, size, margin, out, n);
  }
  /* the piece of the segment within the slabs of the axes where the closest point is inside */
  double tc0 = 0, tc1 = 1;
  for (int j = 0; j < 3; ++j) {
    if (fabs(la[j] + t * d[j]) > size[j] || fabs(d[j]) <= 1e-12) continue;
    double u = (-size[j] - la[j]) / d[j], v = (size[j] - la[j]) / d[j];
    if (u > v) { double x = u; u = v; v = x; }
    tc0 = u > tc0 ? u : tc0;
    tc1 = v < tc1 ? v : tc1;
  }
  if (tc0 > t) tc0 = t;
  if (tc1 < t) tc1 = t;
  double F0 = seg_box_F(la, d, size, tc0), F1 = seg_box_F(la, d, size, tc1);
  double dmin = sqrt(F0 < F1 ? F0 : F1);
  if (t > tc0 && t < tc1 && sqrt(Fbest) < dmin - (1e-6 + 1e-4 * r)) {
    for (int i = 0; i < 3; ++i) p[i] = a[i] + t * (b[i] - a[i]);
    return col_sphere_box(p, r, bpos, bmat, size, margin, out, n);
  }
  for (int i = 0; i < 3; ++i) p[i] = a[i] + tc0 * (b[i] - a[i]);
  n = col_sphere_box(p, r, bpos, bmat, size, margin, out, n);
  if (tc1 > tc0) {
    for (int i = 0; i < 3; ++i) p[i] = a[i] + tc1 * (b[i] - a[i]);
    n = col_sphere_box(p, r, bpos, bmat, size, margin, out, n);
  }
  return n;
}

/* box-box: separating-axis test over the 15 axes (3 + 3 face normals, 9 edge cross products);
 * the least-penetrating axis wins, an edge axis only if it separates clearly more than the best face
 * axis (sep_edge > sep_face + 0.05 |sep_face| + 1e-6).  Face axis: the most anti-parallel face of the
 * other box is clipped against the reference face's four side planes (Sutherland-Hodgman); clipped
 * vertices within margin (up to 8) become contacts at the midpoint to the reference face, in clip
 * order.  Edge axis: one contact between the closest points of the two support edges.  Normal from
 * box 1 to box 2.  Same algorithm as the kernel's box_box (csrc/hip/step.hip). */
static void box_axis(const double* R, int i, double a[3]) { a[0] = R[i]; a[1] = R[3 + i]; a[2] = R[6 + i]; }

static int box_face_clip(const double* pr, const double* Rr, const double* hr, int ir, const double nr[3],
                         const double* pi, const double* Ri, const double* hi, double margin,
                         double pts[8][3], double seps[8]) {
  /* incident face of box i: most anti-parallel to nr */
  int j = 0;
  double best = -1, ax[3];
  for (int k = 0; k < 3; ++k) {
    box_axis(Ri, k, ax);
    double c = fabs(dot3(ax, nr));
    if (c > best) { best = c; j = k; }
  }
  double bj[3], bk[3], bl[3];
  box_axis(Ri, j, bj);
  int k1 = (j + 1) % 3, k2 = (j + 2) % 3;
  box_axis(Ri, k1, bk);
  box_axis(Ri, k2, bl);
  double sgn = dot3(bj, nr) > 0 ? -1.0 : 1.0;  /* outward normal of the incident face faces -nr */
  double poly[8][3], tmp[8][3];
  int np = 4;
  for (int v = 0; v < 4; ++v) {
    double su = (v == 0 || v == 3) ? 1.0 : -1.0, sv = (v < 2) ? 1.0 : -1.0;
    for (int c = 0; c < 3; ++c)
      poly[v][c] = pi[c] + sgn * hi[j] * bj[c] + su * hi[k1] * bk[c] + sv * hi[k2] * bl[c];
  }
  /* reference face: centre and its two in-plane axes */
  double cr[3], ua[3], va[3];
  int r1 = (ir + 1) % 3, r2 = (ir + 2) % 3;
  box_axis(Rr, r1, ua);
  box_axis(Rr, r2, va);
  for (int c = 0; c < 3; ++c) cr[c] = pr[c] + hr[ir] * nr[c];
  for (int side = 0; side < 4; ++side) {
    const double* ax2 = (side < 2) ? ua : va;
    double lim = (side < 2) ? hr[r1] : hr[r2];
    double sg = (side & 1) ? -1.0 : 1.0;  /* keep sg * (x - cr).ax2 <= lim */
    int nn = 0;
    for (int v = 0; v < np; ++v) {
      const double* a = poly[v];
      const double* b = poly[(v + 1) % np];
      double da[3] = {a[0] - cr[0], a[1] - cr[1], a[2] - cr[2]}, db[3] = {b[0] - cr[0], b[1] - cr[1], b[2] - cr[2]};
      double fa = sg * dot3(da, ax2) - lim, fb = sg * dot3(db, ax2) - lim;
      if (fa <= 0) memcpy(tmp[nn++], a, sizeof tmp[0]);
      if ((fa < 0 && fb > 0) || (fa > 0 && fb < 0)) {
        double t = fa / (fa - fb);
        for (int c = 0; c < 3; ++c) tmp[nn][c] = a[c] + t * (b[c] - a[c]);
        ++nn;
      }
    }
    np = nn;
    memcpy(poly, tmp, sizeof poly);
    if (np == 0) return 0;
  }
  int n = 0;
  for (int v = 0; v < np; ++v) {
    double dv[3] = {poly[v][0] - cr[0], poly[v][1] - cr[1], poly[v][2] - cr[2]};
    double sep = dot3(dv, nr);
    if (sep > margin) continue;
    memcpy(pts[n], poly[v], sizeof pts[0]);
    seps[n++] = sep;
  }
  return n;
}

static int col_box_box(const double* p1, const double* R1, const double* h1, const double* p2, const double* R2,
                       const double* h2, double margin, orc_contact* out, int n) {
  double d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double A[3][3], B[3][3];
  for (int i = 0; i < 3; ++i) { box_axis(R1, i, A[i]); box_axis(R2, i, B[i]); }
  double best_face = -1e30, best_edge = -1e30, nf[3] = {0, 0, 0}, ne[3] = {0, 0, 0};
  int face_axis = -1, edge_i = -1, edge_j = -1;
  /* a later face axis must beat the best by more than `tie` (1e-5 of the summed half sizes): two boxes
   * resting face on face have equal separations along both boxes' normals, and rounding alone must not
   * decide which face is the reference (it decides the order of the clipped polygon, which is the
   * Gauss-Seidel row order of the solver) */
  const double tie = 1e-5 * (h1[0] + h1[1] + h1[2] + h2[0] + h2[1] + h2[2]);
  for (int k = 0; k < 15; ++k) {
    double L[3];
    if (k < 3) memcpy(L, A[k], sizeof L);
    else if (k < 6) memcpy(L, B[k - 3], sizeof L);
    else cross3(L, A[(k - 6) / 3], B[(k - 6) % 3]);
    double ln = norm3(L);
    if (ln < 1e-6) continue;  /* parallel edges: covered by the face axes */
    for (int c = 0; c < 3; ++c) L[c] /= ln;
    double ra = 0, rb = 0;
    for (int i = 0; i < 3; ++i) { ra += h1[i] * fabs(dot3(A[i], L)); rb += h2[i] * fabs(dot3(B[i], L)); }
    double s = dot3(d, L);
    double sep = fabs(s) - ra - rb;
    if (sep > margin) return n;
    double sg = s >= 0 ? 1.0 : -1.0;
    if (k < 6) {
      if (sep > best_face + tie) { best_face = sep; face_axis = k; for (int c = 0; c < 3; ++c) nf[c] = sg * L[c]; }
    } else if (sep > best_edge) {
      best_edge = sep; edge_i = (k - 6) / 3; edge_j = (k - 6) % 3;
      for (int c = 0; c < 3; ++c) ne[c] = sg * L[c];
    }
  }
  if (face_axis < 0) return n;
  if (edge_i >= 0 && best_edge > best_face + 0.05 * fabs(best_face) + 1e-6) {
    /* support edges: box 1 towards +ne, box 2 towards -ne, free along A[edge_i] / B[edge_j] */
    double a0[3], a1[3], b0[3], b1[3], c1[3], c2[3];
    for (int c = 0; c < 3; ++c) { a0[c] = p1[c]; b0[c] = p2[c]; }
    for (int i = 0; i < 3; ++i) {
      if (i != edge_i) {
        double sg = dot3(A[i], ne) >= 0 ? 1.0 : -1.0;
        for (int c = 0; c < 3; ++c) a0[c] += sg * h1[i] * A[i][c];
      }
      if (i != edge_j) {
        double sg = dot3(B[i], ne) >= 0 ? -1.0 : 1.0;
        for (int c = 0; c < 3; ++c) b0[c] += sg * h2[i] * B[i][c];
      }
    }
    for (int c = 0; c < 3; ++c) {
      a1[c] = a0[c] + h1[edge_i] * A[edge_i][c]; a0[c] -= h1[edge_i] * A[edge_i][c];
      b1[c] = b0[c] + h2[edge_j] * B[edge_j][c]; b0[c] -= h2[edge_j] * B[edge_j][c];
    }
    segment_segment_closest(a0, a1, b0, b1, c1, c2);
    double pos[3] = {0.5 * (c1[0] + c2[0]), 0.5 * (c1[1] + c2[1]), 0.5 * (c1[2] + c2[2])};
    return add_contact(out, n, best_edge, pos, ne);
  }
  double pts[8][3], seps[8], nr[3];
  int np;
  if (face_axis < 3) {
    np = box_face_clip(p1, R1, h1, face_axis, nf, p2, R2, h2, margin, pts, seps);
    memcpy(nr, nf, sizeof nr);
  } else {
    for (int c = 0; c < 3; ++c) nr[c] = -nf[c];
    np = box_face_clip(p2, R2, h2, face_axis - 3, nr, p1, R1, h1, margin, pts, seps);
  }
  /* every clipped vertex within margin, in clip order (up to 8: the clipped polygon of two faces).
   * Keeping only the deepest few would pick among equal depths by rounding when two faces rest flat
   * on each other, and fp32 / fp64 would pick different corners. */
  for (int v = 0; v < np; ++v) {
    double pos[3];
    for (int c = 0; c < 3; ++c) pos[c] = pts[v][c] - nr[c] * seps[v] / 2;
    n = add_contact(out, n, seps[v], pos, nf);
  }
  return n;
}

/* ---- general convex pairs: ellipsoid, cylinder and mesh geoms (MuJoCo mjc_Convex, which runs
 * libccd's Minkowski Portal Refinement, ccdMPRPenetration, on the two shapes' support functions with
 * each shape inflated by margin/2).  Restated from the published MPR algorithm (Snethen, "XenoCollide",
 * Game Programming Gems 7; libccd mpr.c): portal discovery, portal refinement, then penetration by
 * expanding the portal until the support gain drops under mpr_tolerance (1e-6, mjOption default),
 * at most mpr_iterations (50) expansions.  One contact: dist = margin - depth, normal from geom1 to
 * geom2 (the Minkowski difference is geom1 - geom2), position midway between the two shapes'
 * portal-interpolated surface points.  The device runs the same steps in fp32 (csrc/hip/step.hip
 * mpr_penetration). */
#define MPR_TOL 1e-6
#define MPR_ITER 50
#define MPR_EPS 1e-14
typedef struct {
  int type, nhull;
  const double *pos, *mat, *size, *vert;
  const int* hull;
  double inflate;
} orc_shape;
typedef struct { double v[3], a[3], b[3]; } mpr_point; /* v = a - b: support of geom1 minus geom2 */

static void shape_of(const mrs_model_view* m, orc_ws* w, int g, double margin, orc_shape* s) {
  s->type = m->geom_type[g];
  s->pos = w->geom_xpos + 3 * g;
  s->mat = w->geom_xmat + 9 * g;
  s->size = m->geom_size + 3 * g;
  s->inflate = 0.5 * margin;
  s->vert = NULL; s->hull = NULL; s->nhull = 0;
  if (s->type == MRS_GEOM_MESH) {
    int id = m->geom_dataid[g];
    s->vert = m->mesh_vert + 3 * m->mesh_vertadr[id];
    s->hull = m->mesh_hull + m->mesh_hulladr[id];
    s->nhull = m->mesh_hullnum[id];
  }
}

/* farthest point of the (inflated) shape along dir, world frame */
static void shape_support(const orc_shape* s, const double dir[3], double out[3]) {
  double l[3], p[3] = {0, 0, 0};
  const double* z = s->size;
  matT_vec(l, s->mat, dir);
  switch (s->type) {
    case MRS_GEOM_SPHERE:
    case MRS_GEOM_CAPSULE: {
      double n = norm3(l);
      if (n > MINVAL) for (int i = 0; i < 3; ++i) p[i] = z[0] * l[i] / n;
      if (s->type == MRS_GEOM_CAPSULE) p[2] += l[2] >= 0 ? z[1] : -z[1];
      break;
    }
    case MRS_GEOM_ELLIPSOID: {
      double t[3] = {z[0] * z[0] * l[0], z[1] * z[1] * l[1], z[2] * z[2] * l[2]};
      double den = sqrt(t[0] * l[0] + t[1] * l[1] + t[2] * l[2]);
      if (den > MINVAL) for (int i = 0; i < 3; ++i) p[i] = t[i] / den;
      break;
    }
    case MRS_GEOM_CYLINDER: {
      double rr = sqrt(l[0] * l[0] + l[1] * l[1]);
      if (rr > MINVAL) { p[0] = z[0] * l[0] / rr; p[1] = z[0] * l[1] / rr; }
      p[2] = l[2] >= 0 ? z[1] : -z[1];
      break;
    }
    case MRS_GEOM_BOX:
      for (int i = 0; i < 3; ++i) p[i] = l[i] >= 0 ? z[i] : -z[i];
      break;
    case MRS_GEOM_MESH: {
      double best = -1e300;
      for (int k = 0; k < s->nhull; ++k) {
        const double* v = s->vert + 3 * s->hull[k];
        double d = dot3(v, l);
        if (d > best) { best = d; p[0] = v[0]; p[1] = v[1]; p[2] = v[2]; }
      }
      break;
    }
  }
  mat_vec(out, s->mat, p);
  double dn = norm3(dir);
  for (int i = 0; i < 3; ++i) out[i] += s->pos[i] + (dn > MINVAL ? s->inflate * dir[i] / dn : 0);
}

static void mpr_support(const orc_shape* A, const orc_shape* B, const double dir[3], mpr_point* p) {
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  shape_support(A, dir, p->a);
  shape_support(B, nd, p->b);
  for (int i = 0; i < 3; ++i) p->v[i] = p->a[i] - p->b[i];
}
static void tri_normal(double n[3], const double a[3], const double b[3], const double c[3]) {
  double u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, v[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  cross3(n, u, v);
  normalize3(n);
}
/* closest point to the origin on triangle abc (Ericson, Real-Time Collision Detection 5.1.5) */
static void closest_on_triangle(const double a[3], const double b[3], const double c[3], double out[3]) {
  double ab[3], ac[3], ap[3], bp[3], cp[3];
  for (int i = 0; i < 3; ++i) {
    ab[i] = b[i] - a[i]; ac[i] = c[i] - a[i];
    ap[i] = -a[i]; bp[i] = -b[i]; cp[i] = -c[i];
  }
  double d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) { memcpy(out, a, 3 * sizeof(double)); return; }
  double d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { memcpy(out, b, 3 * sizeof(double)); return; }
  double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    double t = d1 / (d1 - d3);
    for (int i = 0; i < 3; ++i) out[i] = a[i] + t * ab[i];
    return;
  }
  double d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) { memcpy(out, c, 3 * sizeof(double)); return; }
  double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    double t = d2 / (d2 - d6);
    for (int i = 0; i < 3; ++i) out[i] = a[i] + t * ac[i];
    return;
  }
  double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    double t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int i = 0; i < 3; ++i) out[i] = b[i] + t * (c[i] - b[i]);
    return;
  }
  double den = 1 / (va + vb + vc), v = vb * den, ww = vc * den;
  for (int i = 0; i < 3; ++i) out[i] = a[i] + ab[i] * v + ac[i] * ww;
}
/* MPR's penetration vector, the point of the final portal nearest the origin: depth * n (n the portal
 * normal, depth = n.p1) when the origin projects inside the portal, else the nearest edge / vertex
 * point.  Equal to closest_on_triangle; written this way because that formula cancels in fp32 for a
 * long thin portal near the origin, and the device (step.hip mpr_nearest) takes the same branches. */
static void mpr_nearest(const double a[3], const double b[3], const double c[3], double out[3]) {
  double n[3];
  tri_normal(n, a, b, c);
  const double d = dot3(n, a);
  const double q[3] = {d * n[0], d * n[1], d * n[2]};
  const double* V[4] = {a, b, c, a};
  int inside = 1;
  for (int k = 0; k < 3; ++k) {
    double e[3], w[3], x[3];
    for (int i = 0; i < 3; ++i) { e[i] = V[k + 1][i] - V[k][i]; w[i] = q[i] - V[k][i]; }
    cross3(x, e, w);
    if (dot3(x, n) < 0) inside = 0;
  }
  if (inside) { memcpy(out, q, sizeof q); return; }
  closest_on_triangle(a, b, c, out);
}
static void mpr_expand(mpr_point p[4], const mpr_point* v4) {
  double x[3];
  cross3(x, v4->v, p[0].v);
  if (dot3(p[1].v, x) > 0) {
    if (dot3(p[2].v, x) > 0) p[1] = *v4;
    else p[3] = *v4;
  } else {
    if (dot3(p[3].v, x) > 0) p[2] = *v4;
    else p[1] = *v4;
  }
}
static int mpr_reach_tolerance(const mpr_point p[4], const mpr_point* v4, const double n[3]) {
  double d4 = dot3(v4->v, n);
  double g = fmin(d4 - dot3(p[1].v, n), fmin(d4 - dot3(p[2].v, n), d4 - dot3(p[3].v, n)));
  return g <= MPR_TOL;
}
/* 0: origin inside (portal p[0..3] found), 1: touching at p[1], 2: origin on segment p[0]-p[1],
 * -1: separated */
static int mpr_discover(const orc_shape* A, const orc_shape* B, mpr_point p[4]) {
  for (int i = 0; i < 3; ++i) { p[0].a[i] = A->pos[i]; p[0].b[i] = B->pos[i]; p[0].v[i] = A->pos[i] - B->pos[i]; }
  if (dot3(p[0].v, p[0].v) < 1e-20) p[0].v[0] += 1e-5;
  double dir[3] = {-p[0].v[0], -p[0].v[1], -p[0].v[2]};
  normalize3(dir);
  mpr_support(A, B, dir, &p[1]);
  if (dot3(p[1].v, dir) <= 0) return -1;
  cross3(dir, p[0].v, p[1].v);
  if (dot3(dir, dir) < MPR_EPS) return dot3(p[1].v, p[1].v) < MPR_EPS ? 1 : 2;
  normalize3(dir);
  mpr_support(A, B, dir, &p[2]);
  if (dot3(p[2].v, dir) <= 0) return -1;
  double va[3], vb[3];
  for (int i = 0; i < 3; ++i) { va[i] = p[1].v[i] - p[0].v[i]; vb[i] = p[2].v[i] - p[0].v[i]; }
  cross3(dir, va, vb);
  normalize3(dir);
  if (dot3(dir, p[0].v) > 0) {
    mpr_point t = p[1]; p[1] = p[2]; p[2] = t;
    for (int i = 0; i < 3; ++i) dir[i] = -dir[i];
  }
  for (int it = 0; it < MPR_ITER; ++it) {
    mpr_support(A, B, dir, &p[3]);
    if (dot3(p[3].v, dir) <= 0) return -1;
    double x[3];
    int replaced = 0;
    cross3(x, p[1].v, p[3].v);
    if (dot3(x, p[0].v) < -MPR_EPS) { p[2] = p[3]; replaced = 1; }
    else {
      cross3(x, p[3].v, p[2].v);
      if (dot3(x, p[0].v) < -MPR_EPS) { p[1] = p[3]; replaced = 1; }
    }
    if (!replaced) return 0;
    for (int i = 0; i < 3; ++i) { va[i] = p[1].v[i] - p[0].v[i]; vb[i] = p[2].v[i] - p[0].v[i]; }
    cross3(dir, va, vb);
    normalize3(dir);
  }
  return 0;
}
static void mpr_position(const mpr_point p[4], double pos[3]) {
  double n[3], x[3], b[4];
  tri_normal(n, p[1].v, p[2].v, p[3].v);
  cross3(x, p[1].v, p[2].v); b[0] = dot3(x, p[3].v);
  cross3(x, p[3].v, p[2].v); b[1] = dot3(x, p[0].v);
  cross3(x, p[0].v, p[1].v); b[2] = dot3(x, p[3].v);
  cross3(x, p[2].v, p[1].v); b[3] = dot3(x, p[0].v);
  double sum = b[0] + b[1] + b[2] + b[3];
  if (sum <= MPR_EPS) {
    b[0] = 0;
    cross3(x, p[2].v, p[3].v); b[1] = dot3(x, n);
    cross3(x, p[3].v, p[1].v); b[2] = dot3(x, n);
    cross3(x, p[1].v, p[2].v); b[3] = dot3(x, n);
    sum = b[1] + b[2] + b[3];
  }
  for (int i = 0; i < 3; ++i) {
    double pa = 0, pb = 0;
    for (int k = 0; k < 4; ++k) { pa += b[k] * p[k].a[i]; pb += b[k] * p[k].b[i]; }
    pos[i] = 0.5 * (pa + pb) / sum;
  }
}
/* returns 1 with depth (of the inflated shapes), unit normal (geom1 -> geom2) and position */
static int mpr_penetration(const orc_shape* A, const orc_shape* B, double* depth, double nrm[3], double pos[3]) {
  mpr_point p[4], v4;
  int r = mpr_discover(A, B, p);
  if (r < 0 || r == 1) return 0;
  if (r == 2) {
    for (int i = 0; i < 3; ++i) { nrm[i] = p[1].v[i]; pos[i] = 0.5 * (p[1].a[i] + p[1].b[i]); }
    *depth = normalize3(nrm);
    return 1;
  }
  /* refinement: expand until the portal holds the origin */
  for (int it = 0;; ++it) {
    double n[3];
    tri_normal(n, p[1].v, p[2].v, p[3].v);
    if (dot3(n, p[1].v) >= 0) break;
    mpr_support(A, B, n, &v4);
    if (dot3(v4.v, n) < 0 || mpr_reach_tolerance(p, &v4, n) || it >= MPR_ITER) return 0;
    mpr_expand(p, &v4);
  }
  /* penetration: expand towards the surface of the Minkowski difference nearest the portal */
  for (int it = 0;; ++it) {
    double n[3];
    tri_normal(n, p[1].v, p[2].v, p[3].v);
    mpr_support(A, B, n, &v4);
    if (mpr_reach_tolerance(p, &v4, n) || it > MPR_ITER) {
      mpr_nearest(p[1].v, p[2].v, p[3].v, nrm);
      *depth = normalize3(nrm);
      if (*depth < MINVAL) return 0;
      mpr_position(p, pos);
      return 1;
    }
    mpr_expand(p, &v4);
  }
}
/* ---- MPR contact polish: the exact penetration direction next to MPR's answer (the minimum
 * translation that EPA, MuJoCo 3.3's native convex collision, converges to; libccd's MPR measures the
 * depth along its portal direction, which on elongated shapes can be millimetres deeper).
 * MPR stops once the portal is within mpr_tolerance of the surface of A - B; on a curved surface the
 * portal's normal is then fixed only to ~sqrt(2 tol / r) (7e-3 rad at r = 4 cm), and which portal fp32
 * and fp64 stop on differs.  The penetration direction itself is well defined: the minimiser over unit
 * n of the support function of A - B, h(n) = h_A(n) + h_B(-n) (its minimum is the depth), a convex
 * problem on the sphere whose solution lies next to MPR's normal.  Each shape is split into a
 * polyhedral part (vertices: mesh hull, box corners, capsule segment ends, sphere / ellipsoid centre;
 * for B the vertices of -B) and a smooth part (sphere radius and margin/2 inflation, ellipsoid), so
 *   h(n) = max_i a_i.n + max_j b'_j.n + h_S(n),  b' = -b,  h_S = (R_A + R_B)|n| + h_EA(n) + h_EB(n).
 * Active-set Newton from MPR's normal: the active vertices of each polyhedral part (vertex, edge, face)
 * give the constraints (v_k - v_0).n = 0, Newton on the sphere within them uses the smooth part's
 * curvature (2-D in the tangent plane; 1-D on the great circle of an edge; none for a face or two skew
 * edges, whose normal n then is); a step stops where another vertex becomes active (added), and at the
 * solution the multipliers -- the convex weights of the feature's vertices that make the tangential
 * gradient vanish -- must be feasible, else the vertex with the negative weight is dropped.  Pairs
 * without a curved shape (polytope pairs: MPR's portal lies on a face), cylinders (a disk rim is not
 * smooth), and any iteration that does not settle keep MPR's contact.  Position: midway between the
 * shapes' contact points (smooth support + the feature point of the weights).  Same steps in fp32 on
 * the device (csrc/hip/step.hip mpr_polish). */
#define POL_MAXV 4
#define POL_PASSES 12
#define POL_NEWTON 12
typedef struct {
  int nv, mesh, ell;
  double v[8][3];                       /* vertices of the part (non-mesh), world, sign applied */
  const double *vert, *pos, *mat;       /* mesh hull vertices (local) */
  const int* hull;
  double sgn, R, M[9];                  /* sign (+1 A, -1 B), sphere radius, ellipsoid R diag(a^2) R' */
} pol_part;

static int pol_part_of(const orc_shape* s, double sgn, pol_part* p) {
  memset(p, 0, sizeof *p);
  p->sgn = sgn;
  p->R = s->inflate;
  const double* z = s->size;
  double c[3] = {s->pos[0], s->pos[1], s->pos[2]};
  switch (s->type) {
    case MRS_GEOM_SPHERE:
      p->nv = 1; p->R += z[0];
      for (int i = 0; i < 3; ++i) p->v[0][i] = sgn * c[i];
      return 1;
    case MRS_GEOM_CAPSULE:
      p->nv = 2; p->R += z[0];
      for (int i = 0; i < 3; ++i) {
        p->v[0][i] = sgn * (c[i] - s->mat[3 * i + 2] * z[1]);
        p->v[1][i] = sgn * (c[i] + s->mat[3 * i + 2] * z[1]);
      }
      return 1;
    case MRS_GEOM_ELLIPSOID:
      p->nv = 1; p->ell = 1;
      for (int i = 0; i < 3; ++i) p->v[0][i] = sgn * c[i];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          double v = 0;
          for (int k = 0; k < 3; ++k) v += s->mat[3 * i + k] * z[k] * z[k] * s->mat[3 * j + k];
          p->M[3 * i + j] = v;
        }
      return 1;
    case MRS_GEOM_BOX:
      p->nv = 8;
      for (int k = 0; k < 8; ++k) {
        double l[3] = {(k & 1) ? z[0] : -z[0], (k & 2) ? z[1] : -z[1], (k & 4) ? z[2] : -z[2]}, x[3];
        mat_vec(x, s->mat, l);
        for (int i = 0; i < 3; ++i) p->v[k][i] = sgn * (c[i] + x[i]);
      }
      return 1;
    case MRS_GEOM_MESH:
      p->nv = s->nhull; p->mesh = 1;
      p->vert = s->vert; p->hull = s->hull; p->pos = s->pos; p->mat = s->mat;
      return 1;
    default:
      return 0;  /* cylinder: not polished */
  }
}
static void pol_vertex(const pol_part* p, int k, double out[3]) {
  if (!p->mesh) { for (int i = 0; i < 3; ++i) out[i] = p->v[k][i]; return; }
  double x[3];
  mat_vec(x, p->mat, p->vert + 3 * p->hull[k]);
  for (int i = 0; i < 3; ++i) out[i] = p->sgn * (p->pos[i] + x[i]);
}
/* smooth part of one shape (of -B for B): support along n and curvature Hessian (added into H) */
static void pol_smooth(const pol_part* p, const double n[3], double s[3], double H[9]) {
  for (int i = 0; i < 3; ++i) s[i] = p->R * n[i];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) H[3 * i + j] += p->R * ((i == j) - n[i] * n[j]);
  if (p->ell) {
    double Mn[3];
    mat_vec(Mn, p->M, n);
    double h = sqrt(dot3(n, Mn));
    if (h < MINVAL) return;
    for (int i = 0; i < 3; ++i) s[i] += Mn[i] / h;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) H[3 * i + j] += (p->M[3 * i + j] - Mn[i] * Mn[j] / (h * h)) / h;
  }
}
typedef struct { const pol_part* P[2]; int F[2][POL_MAXV], nf[2]; } pol_state;

/* gradient G = s_S(n) + v_A0 + v_B0 and Hessian of the smooth part at n */
static void pol_grad(const pol_state* st, const double n[3], double G[3], double H[9], double sS[2][3]) {
  memset(H, 0, 9 * sizeof(double));
  for (int i = 0; i < 3; ++i) G[i] = 0;
  for (int q = 0; q < 2; ++q) {
    double v0[3];
    pol_smooth(st->P[q], n, sS[q], H);
    pol_vertex(st->P[q], st->F[q][0], v0);
    for (int i = 0; i < 3; ++i) G[i] += sS[q][i] + v0[i];
  }
}
/* orthonormal basis of the feature constraint vectors (v_k - v_0); returns the rank (<= 3) */
static int pol_basis(const pol_state* st, double Q[3][3]) {
  int r = 0;
  for (int q = 0; q < 2; ++q) {
    double v0[3];
    pol_vertex(st->P[q], st->F[q][0], v0);
    for (int k = 1; k < st->nf[q]; ++k) {
      double e[3];
      pol_vertex(st->P[q], st->F[q][k], e);
      for (int i = 0; i < 3; ++i) e[i] -= v0[i];
      double len = norm3(e);
      for (int j = 0; j < r; ++j) {
        double d = dot3(e, Q[j]);
        for (int i = 0; i < 3; ++i) e[i] -= d * Q[j][i];
      }
      double el = norm3(e);
      if (el <= 1e-9 * len || len < MINVAL) continue;
      if (r == 3) return 4;
      for (int i = 0; i < 3; ++i) Q[r][i] = e[i] / el;
      ++r;
    }
  }
  return r;
}
static void pol_tangent(const double n[3], double t1[3], double t2[3]) {
  double a[3] = {0, 0, 0};
  a[fabs(n[0]) < 0.6 ? 0 : (fabs(n[1]) < 0.6 ? 1 : 2)] = 1;
  double d = dot3(a, n);
  for (int i = 0; i < 3; ++i) t1[i] = a[i] - d * n[i];
  normalize3(t1);
  cross3(t2, n, t1);
}
/* move n -> normalize(n + dl), stopping at the first vertex that ties with its part's active
 * vertices; returns 1 when a vertex was added (n moved to the tie), 0 when the full step was taken,
 * -1 when a feature is full */
static int pol_move(pol_state* st, double n[3], const double dl[3]) {
  double tmin = 1;
  int qmin = -1, kmin = -1;
  for (int q = 0; q < 2; ++q) {
    const pol_part* P = st->P[q];
    double v0[3];
    pol_vertex(P, st->F[q][0], v0);
    const double c0 = dot3(v0, n), d0 = dot3(v0, dl);
    for (int k = 0; k < P->nv; ++k) {
      int in = 0;
      for (int f = 0; f < st->nf[q]; ++f) in |= st->F[q][f] == k;
      if (in) continue;
      double v[3];
      pol_vertex(P, k, v);
      const double c = dot3(v, n) - c0, d = dot3(v, dl) - d0;
      if (c + d <= 0 || d <= 0) continue;
      double t = -c / d;
      if (t < 0) t = 0;
      if (t < tmin) { tmin = t; qmin = q; kmin = k; }
    }
  }
  for (int i = 0; i < 3; ++i) n[i] += tmin * dl[i];
  normalize3(n);
  if (qmin < 0) return 0;
  if (st->nf[qmin] >= POL_MAXV) return -1;
  st->F[qmin][st->nf[qmin]++] = kmin;
  return 1;
}
static void pol_drop(pol_state* st, int q, int f) {
  for (int k = f; k + 1 < st->nf[q]; ++k) st->F[q][k] = st->F[q][k + 1];
  --st->nf[q];
}
/* convex weights of the feature vertices (beyond each part's anchor) that make the tangential
 * gradient vanish; returns 1 feasible (w filled, per part, for vertices 1..nf-1), 0 after dropping a
 * vertex, -1 when the case is not handled */
static int pol_kkt(pol_state* st, const double n[3], const double G[3], double w[2][POL_MAXV]) {
  double t1[3], t2[3];
  pol_tangent(n, t1, t2);
  int m = st->nf[0] + st->nf[1] - 2;
  memset(w, 0, 2 * POL_MAXV * sizeof(double));
  if (m == 0) return 1;
  /* columns: the constraint vectors, tangential components */
  double E[6][2];
  int cq[6], cf[6], nc = 0;
  for (int q = 0; q < 2; ++q) {
    double v0[3];
    pol_vertex(st->P[q], st->F[q][0], v0);
    for (int f = 1; f < st->nf[q]; ++f) {
      double e[3];
      pol_vertex(st->P[q], st->F[q][f], e);
      for (int i = 0; i < 3; ++i) e[i] -= v0[i];
      E[nc][0] = dot3(e, t1); E[nc][1] = dot3(e, t2);
      cq[nc] = q; cf[nc] = f; ++nc;
    }
  }
  const double g1 = dot3(G, t1), g2 = dot3(G, t2);
  if (m == 1) {
    const double el = sqrt(E[0][0] * E[0][0] + E[0][1] * E[0][1]);
    if (el < MINVAL) return -1;
    const double x = -(g1 * E[0][0] + g2 * E[0][1]) / (el * el);
    if (x < 0) { pol_drop(st, cq[0], cf[0]); return 0; }
    if (x > 1) { pol_drop(st, cq[0], 0); return 0; }
    w[cq[0]][cf[0]] = x;
    return 1;
  }
  if (m == 2) {
    const double det = E[0][0] * E[1][1] - E[1][0] * E[0][1];
    if (fabs(det) < MINVAL) return -1;
    const double x0 = (-g1 * E[1][1] + g2 * E[1][0]) / det, x1 = (-g2 * E[0][0] + g1 * E[0][1]) / det;
    if (cq[0] == cq[1]) {  /* a triangle of one part: barycentric (1 - x0 - x1, x0, x1) */
      const double x2 = 1 - x0 - x1;
      const double worst = fmin(x2, fmin(x0, x1));
      if (worst < 0) {
        pol_drop(st, cq[0], worst == x0 ? cf[0] : (worst == x1 ? cf[1] : 0));
        return 0;
      }
    } else {               /* an edge of each part */
      const double v0 = fmin(x0, 1 - x0), v1 = fmin(x1, 1 - x1);
      if (v0 < 0 || v1 < 0) {
        const int c = v0 <= v1 ? 0 : 1;
        const double x = c == 0 ? x0 : x1;
        pol_drop(st, cq[c], x < 0 ? cf[c] : 0);
        return 0;
      }
    }
    w[cq[0]][cf[0]] = x0;
    w[cq[1]][cf[1]] = x1;
    return 1;
  }
  if (m == 3 && (st->nf[0] == 1 || st->nf[1] == 1)) {
    /* a coplanar quad of one part: the point lies in one of its triangles (Caratheodory) */
    const int q = cq[0];
    for (int a = 0; a < 3; ++a)
      for (int b = a + 1; b < 3; ++b) {
        /* triangle (anchor, a, b) */
        const double det = E[a][0] * E[b][1] - E[b][0] * E[a][1];
        if (fabs(det) < MINVAL) continue;
        const double x0 = (-g1 * E[b][1] + g2 * E[b][0]) / det, x1 = (-g2 * E[a][0] + g1 * E[a][1]) / det;
        if (x0 >= 0 && x1 >= 0 && x0 + x1 <= 1) { w[q][cf[a]] = x0; w[q][cf[b]] = x1; return 1; }
      }
    /* triangle (a, b, c) without the anchor: x_a + x_b + x_c = 1 */
    {
      const double det = E[1][0] * E[2][1] - E[2][0] * E[1][1] - (E[0][0] * E[2][1] - E[2][0] * E[0][1]) +
                         (E[0][0] * E[1][1] - E[1][0] * E[0][1]);
      if (fabs(det) > MINVAL) {
        /* solve [E0 E1 E2; 1 1 1] x = [-g; 1] by Cramer */
        double A3[9] = {E[0][0], E[1][0], E[2][0], E[0][1], E[1][1], E[2][1], 1, 1, 1}, rhs[3] = {-g1, -g2, 1}, x[3];
        for (int c = 0; c < 3; ++c) {
          double B3[9];
          memcpy(B3, A3, sizeof B3);
          for (int r = 0; r < 3; ++r) B3[3 * r + c] = rhs[r];
          x[c] = (B3[0] * (B3[4] * B3[8] - B3[5] * B3[7]) - B3[1] * (B3[3] * B3[8] - B3[5] * B3[6]) +
                  B3[2] * (B3[3] * B3[7] - B3[4] * B3[6])) /
                 (A3[0] * (A3[4] * A3[8] - A3[5] * A3[7]) - A3[1] * (A3[3] * A3[8] - A3[5] * A3[6]) +
                  A3[2] * (A3[3] * A3[7] - A3[4] * A3[6]));
        }
        if (x[0] >= 0 && x[1] >= 0 && x[2] >= 0) {
          w[q][cf[0]] = x[0]; w[q][cf[1]] = x[1]; w[q][cf[2]] = x[2];
          return 1;
        }
      }
    }
    return -1;
  }
  return -1;
}
/* returns 1 with the polished depth / normal / position, 0 to keep MPR's */
static int pol_debug = -1;
#define POL_FAIL(c)                                                                        \
  do {                                                                                     \
    if (pol_debug < 0) pol_debug = getenv("ORC_POLISH_DEBUG") != NULL;                     \
    if (pol_debug) fprintf(stderr, "polish fallback %d (types %d %d)\n", c, A->type, B->type); \
    return 0;                                                                              \
  } while (0)
static int mpr_polish(const orc_shape* A, const orc_shape* B, const double n0[3], double mpr_depth, double* depth,
                      double nrm[3], double pos[3]) {
  if (A->type == MRS_GEOM_CYLINDER || B->type == MRS_GEOM_CYLINDER) POL_FAIL(1);
  const int curvedA = A->type == MRS_GEOM_SPHERE || A->type == MRS_GEOM_CAPSULE || A->type == MRS_GEOM_ELLIPSOID;
  const int curvedB = B->type == MRS_GEOM_SPHERE || B->type == MRS_GEOM_CAPSULE || B->type == MRS_GEOM_ELLIPSOID;
  if (!curvedA && !curvedB) POL_FAIL(2);
  pol_part PA, PB;
  if (!pol_part_of(A, 1, &PA) || !pol_part_of(B, -1, &PB)) POL_FAIL(3);
  pol_state st;
  st.P[0] = &PA; st.P[1] = &PB;
  double n[3] = {n0[0], n0[1], n0[2]};
  for (int q = 0; q < 2; ++q) {
    double best = -1e300;
    st.nf[q] = 1;
    for (int k = 0; k < st.P[q]->nv; ++k) {
      double v[3];
      pol_vertex(st.P[q], k, v);
      const double d = dot3(v, n);
      if (d > best) { best = d; st.F[q][0] = k; }
    }
  }
  double G[3], H[9], sS[2][3], w[2][POL_MAXV];
  int done = 0;
  for (int pass = 0; pass < POL_PASSES && !done; ++pass) {
    double Q[3][3];
    const int rank = pol_basis(&st, Q);
    if (rank > 2) {
      /* the step stopped where a third independent vertex tied: n is fixed by any two of the
       * constraints; accept the first single-vertex drop whose feature is optimal at n */
      pol_grad(&st, n, G, H, sS);
      int found = 0;
      for (int q = 0; q < 2 && !found; ++q)
        for (int f = 0; f < st.nf[q] && !found; ++f) {
          pol_state t = st;
          pol_drop(&t, q, f);
          double Qt[3][3];
          if (pol_basis(&t, Qt) != 2) continue;
          double Gt[3], Ht[9], sSt[2][3];
          pol_grad(&t, n, Gt, Ht, sSt);
          if (pol_kkt(&t, n, Gt, w) == 1) { st = t; found = 1; memcpy(G, Gt, sizeof Gt); memcpy(sS, sSt, sizeof sSt); }
        }
      if (!found) POL_FAIL(4);
      done = 1;
      break;
    }
    int moved = 0, conv = 0;
    if (rank == 2) {
      double t[3], dl[3];
      cross3(t, Q[0], Q[1]);
      normalize3(t);
      if (dot3(t, n) < 0) for (int i = 0; i < 3; ++i) t[i] = -t[i];
      for (int i = 0; i < 3; ++i) dl[i] = t[i] - n[i];
      const int r = pol_move(&st, n, dl);
      if (r < 0) POL_FAIL(5);
      moved = r;
      conv = !r;
    } else {
      for (int it = 0; it < POL_NEWTON; ++it) {
        pol_grad(&st, n, G, H, sS);
        const double lam = dot3(G, n);
        double dl[3];
        if (rank == 0) {
          double t1[3], t2[3], Ht1[3], Ht2[3];
          pol_tangent(n, t1, t2);
          mat_vec(Ht1, H, t1);
          mat_vec(Ht2, H, t2);
          const double a11 = dot3(t1, Ht1) - lam, a22 = dot3(t2, Ht2) - lam, a12 = dot3(t1, Ht2);
          const double det = a11 * a22 - a12 * a12;
          if (!(a11 > 0 && det > 0)) POL_FAIL(6);
          const double b1 = -dot3(G, t1), b2 = -dot3(G, t2);
          const double x1 = (b1 * a22 - b2 * a12) / det, x2 = (b2 * a11 - b1 * a12) / det;
          for (int i = 0; i < 3; ++i) dl[i] = x1 * t1[i] + x2 * t2[i];
        } else {
          /* great circle orthogonal to Q[0] through n */
          double d = dot3(n, Q[0]);
          for (int i = 0; i < 3; ++i) n[i] -= d * Q[0][i];
          normalize3(n);
          pol_grad(&st, n, G, H, sS);
          const double lm = dot3(G, n);
          double t[3], Ht[3];
          cross3(t, Q[0], n);
          mat_vec(Ht, H, t);
          const double f2 = dot3(t, Ht) - lm;
          if (!(f2 > 0)) POL_FAIL(7);
          const double th = -dot3(G, t) / f2;
          for (int i = 0; i < 3; ++i) dl[i] = th * t[i];
        }
        const double step = norm3(dl);
        const int r = pol_move(&st, n, dl);
        if (r < 0) POL_FAIL(8);
        if (r > 0) { moved = 1; break; }
        if (step < 1e-13) { conv = 1; break; }
      }
    }
    if (moved) continue;
    if (!conv) POL_FAIL(9);
    pol_grad(&st, n, G, H, sS);
    const int k = pol_kkt(&st, n, G, w);
    if (k < 0) POL_FAIL(10);
    done = k == 1;
  }
  if (!done) POL_FAIL(11);
  /* sanity: next to MPR's answer */
  double dp = dot3(G, n);
  /* a local minimiser next to MPR's normal, never deeper than MPR's portal distance (MPR measures
   * along the direction its portal search found, the polish minimises over directions) */
  if (dot3(n, n0) < 0.8 || !(dp > 0) || dp > mpr_depth + MPR_TOL) POL_FAIL(12);
  double pA[3], pB[3], v0[3], e[3];
  for (int q = 0; q < 2; ++q) {
    double* pt = q ? pB : pA;
    pol_vertex(st.P[q], st.F[q][0], v0);
    for (int i = 0; i < 3; ++i) pt[i] = v0[i] + sS[q][i];
    for (int f = 1; f < st.nf[q]; ++f) {
      pol_vertex(st.P[q], st.F[q][f], e);
      for (int i = 0; i < 3; ++i) pt[i] += w[q][f] * (e[i] - v0[i]);
    }
  }
  *depth = dp;
  for (int i = 0; i < 3; ++i) { nrm[i] = n[i]; pos[i] = 0.5 * (pA[i] - pB[i]); }
  return 1;
}

/* ---- face contacts of two polytopes (box and mesh pairs, at least one mesh): this restatement of
 * MuJoCo's multi-contact convex collision (multiccd) [restated; verify against upstream].  MPR gives
 * the contact normal n (geom1 -> geom2).  Each shape's support face is the face whose outward normal
 * is nearest n (geom1) or -n (geom2): a box face, or a polygon of the mesh's hull (mesh_poly*).  When
 * the better aligned of the two is within POLY_COS of n (a face contact), it is the reference face and
 * the other the incident face: the incident polygon is clipped by the reference polygon's side planes
 * (Sutherland-Hodgman, in the incident polygon's vertex order), and every clipped vertex within margin
 * of the reference plane is a contact (at most 8, in clip order): distance d to the reference plane,
 * position midway between the vertex and the plane, normal the reference face's (geom1 -> geom2).  A
 * flat face-on-face rest gets its corners, a box tipped onto an edge the edge's ends.  Otherwise
 * (edge-edge, vertex contacts) MPR's single contact stays.  The reference face is geom1's unless
 * geom2's alignment is larger by more than 1e-4 (fp32 and fp64 break a tie between two flat faces
 * the same way).  Faces of more than POLY_MAXV vertices keep MPR's single contact, as on the device. */
#define POLY_MAXV 8
#define POLY_COS 0.999
typedef struct { int n; double v[POLY_MAXV][3]; double nrm[3]; } orc_poly;
/* support face of shape s (box or mesh geom g) along dir; returns the alignment n_face.dir, or -2
 * when the face has more than POLY_MAXV vertices */
static double poly_support_face(const mrs_model_view* m, const orc_shape* s, int g, const double dir[3], orc_poly* f) {
  const double* R = s->mat;
  if (s->type == MRS_GEOM_BOX) {
    double l[3];
    matT_vec(l, R, dir);
    int ax = 0;
    for (int i = 1; i < 3; ++i)
      if (fabs(l[i]) > fabs(l[ax])) ax = i;
    const double sg = l[ax] >= 0 ? 1.0 : -1.0;
    const int j = (ax + 1) % 3, k = (ax + 2) % 3;
    /* corners counter-clockwise about the outward normal sg e_ax: (j, k) signs (-,-), (+,-), (+,+),
     * (-,+) about +e_ax (e_j x e_k = e_ax), reversed about -e_ax */
    static const double cj[4] = {-1, 1, 1, -1}, ck[4] = {-1, -1, 1, 1};
    f->n = 4;
    for (int q = 0; q < 4; ++q) {
      const int qq = sg > 0 ? q : 3 - q;
      double lp[3];
      lp[ax] = sg * s->size[ax];
      lp[j] = cj[qq] * s->size[j];
      lp[k] = ck[qq] * s->size[k];
      double wv[3];
      mat_vec(wv, R, lp);
      for (int i = 0; i < 3; ++i) f->v[q][i] = s->pos[i] + wv[i];
    }
    for (int i = 0; i < 3; ++i) f->nrm[i] = sg * R[3 * i + ax];
    return fabs(l[ax]);
  }
  const int id = m->geom_dataid[g];
  int best = -1;
  double ba = -3;
  for (int q = m->mesh_polyadr[id]; q < m->mesh_polyadr[id] + m->mesh_polynum[id]; ++q) {
    double nw[3];
    mat_vec(nw, R, m->mesh_polynormal + 3 * q);
    const double a = dot3(nw, dir);
    if (a > ba) { ba = a; best = q; }
  }
  if (best < 0 || m->mesh_polyvertnum[best] > POLY_MAXV) return -2;
  mat_vec(f->nrm, R, m->mesh_polynormal + 3 * best);
  f->n = m->mesh_polyvertnum[best];
  const double* vb = m->mesh_vert + 3 * m->mesh_vertadr[id];
  for (int q = 0; q < f->n; ++q) {
    double wv[3];
    mat_vec(wv, R, vb + 3 * m->mesh_polyvert[m->mesh_polyvertadr[best] + q]);
    for (int i = 0; i < 3; ++i) f->v[q][i] = s->pos[i] + wv[i];
  }
  return ba;
}
static int col_poly_faces(const mrs_model_view* m, const orc_shape* A, int g1, const orc_shape* B, int g2,
                          const double nrm[3], double margin, orc_contact* out, int n) {
  orc_poly fa, fb;
  const double nb[3] = {-nrm[0], -nrm[1], -nrm[2]};
  const double aa = poly_support_face(m, A, g1, nrm, &fa), ab = poly_support_face(m, B, g2, nb, &fb);
  if (aa < -1 || ab < -1) return -1;
  const int refA = !(ab > aa + 1e-4);
  if ((refA ? aa : ab) < POLY_COS) return -1;
  const orc_poly* ref = refA ? &fa : &fb;
  const orc_poly* inc = refA ? &fb : &fa;
  double buf[2][2 * POLY_MAXV][3];
  int cnt = inc->n, cur = 0;
  for (int q = 0; q < cnt; ++q)
    for (int i = 0; i < 3; ++i) buf[0][q][i] = inc->v[q][i];
  for (int e = 0; e < ref->n && cnt > 0; ++e) {
    const double* r0 = ref->v[e];
    const double* r1 = ref->v[(e + 1) % ref->n];
    const double ed[3] = {r1[0] - r0[0], r1[1] - r0[1], r1[2] - r0[2]};
    double h[3];
    cross3(h, ref->nrm, ed); /* inward side normal of the edge */
    int out_n = 0;
    for (int q = 0; q < cnt; ++q) {
      const double* pc = buf[cur][q];
      const double* pn = buf[cur][(q + 1) % cnt];
      const double dc = (pc[0] - r0[0]) * h[0] + (pc[1] - r0[1]) * h[1] + (pc[2] - r0[2]) * h[2];
      const double dn = (pn[0] - r0[0]) * h[0] + (pn[1] - r0[1]) * h[1] + (pn[2] - r0[2]) * h[2];
      if (dc >= 0 && out_n < 2 * POLY_MAXV)
        for (int i = 0; i < 3; ++i) buf[1 - cur][out_n][i] = pc[i];
      if (dc >= 0) ++out_n;
      if ((dc >= 0) != (dn >= 0) && out_n < 2 * POLY_MAXV) {
        const double t = dc / (dc - dn);
        for (int i = 0; i < 3; ++i) buf[1 - cur][out_n][i] = pc[i] + t * (pn[i] - pc[i]);
        ++out_n;
      }
    }
    cnt = out_n < 2 * POLY_MAXV ? out_n : 2 * POLY_MAXV;
    cur = 1 - cur;
  }
  const double sg = refA ? 1.0 : -1.0;
  const double cn[3] = {sg * ref->nrm[0], sg * ref->nrm[1], sg * ref->nrm[2]};
  const int n0 = n;
  for (int q = 0; q < cnt; ++q) {
    const double* p = buf[cur][q];
    const double d = (p[0] - ref->v[0][0]) * ref->nrm[0] + (p[1] - ref->v[0][1]) * ref->nrm[1] +
                     (p[2] - ref->v[0][2]) * ref->nrm[2];
    if (d > margin) continue;
    double pos[3];
    for (int i = 0; i < 3; ++i) pos[i] = p[i] - 0.5 * d * ref->nrm[i];
    n = add_contact(out, n, d, pos, cn);
  }
  return n > n0 ? n : -1;
}
static int col_convex(const mrs_model_view* m, orc_ws* w, int g1, int g2, double margin, orc_contact* out, int n) {
  orc_shape A, B;
  shape_of(m, w, g1, margin, &A);
  shape_of(m, w, g2, margin, &B);
  double depth, nrm[3], pos[3];
  if (!mpr_penetration(&A, &B, &depth, nrm, pos)) return n;
  {
    /* two polytopes, at least one a mesh: the face contacts, when the contact is face-on */
    const int p1 = A.type == MRS_GEOM_BOX || A.type == MRS_GEOM_MESH, p2 = B.type == MRS_GEOM_BOX || B.type == MRS_GEOM_MESH;
    if (p1 && p2 && (A.type == MRS_GEOM_MESH || B.type == MRS_GEOM_MESH) && !(m->restate & MRS_RESTATE_NO_MULTICCD)) {
      const int r = col_poly_faces(m, &A, g1, &B, g2, nrm, margin, out, n);
      if (r >= 0) return r;
    }
  }
  static int no_polish = -1;  /* diagnostics: ORC_NO_POLISH=1 keeps MPR's contact (scripts/diag_mpr.py) */
  if (no_polish < 0) no_polish = getenv("ORC_NO_POLISH") != NULL;
  if (!no_polish && !(m->restate & MRS_RESTATE_NO_MPR_POLISH)) mpr_polish(&A, &B, nrm, depth, &depth, nrm, pos);
  return add_contact(out, n, margin - depth, pos, nrm);
}
/* plane (geom1) vs ellipsoid: the support point along -normal (mjc_PlaneEllipsoid) */
static int col_plane_convex_support(const mrs_model_view* m, orc_ws* w, const double* ppos, const double* pmat,
                                    int g2, double margin, orc_contact* out, int n) {
  orc_shape B;
  shape_of(m, w, g2, 0, &B);
  double nrm[3] = {pmat[2], pmat[5], pmat[8]}, nd[3] = {-nrm[0], -nrm[1], -nrm[2]}, s[3];
  shape_support(&B, nd, s);
  double dv[3] = {s[0] - ppos[0], s[1] - ppos[1], s[2] - ppos[2]};
  double dist = dot3(dv, nrm);
  if (dist > margin) return n;
  double pos[3];
  for (int i = 0; i < 3; ++i) pos[i] = s[i] - nrm[i] * dist / 2;
  return add_contact(out, n, dist, pos, nrm);
}
/* plane vs cylinder (after mjc_PlaneCylinder): on each cap the rim point deepest along -normal, and
 * on the deeper cap the two rim points at +-120 degrees from it (a resting cylinder stands on a
 * triangle); the rim direction falls back to the cylinder's x axis when the axis is parallel to the
 * normal */
static int col_plane_cylinder(const double* ppos, const double* pmat, const double* cpos, const double* cmat,
                              const double* size, double margin, orc_contact* out, int n) {
  double nrm[3] = {pmat[2], pmat[5], pmat[8]}, ax[3] = {cmat[2], cmat[5], cmat[8]};
  double an = dot3(ax, nrm), d[3];
  for (int i = 0; i < 3; ++i) d[i] = -nrm[i] + an * ax[i];
  if (dot3(d, d) < 1e-12) { d[0] = cmat[0]; d[1] = cmat[3]; d[2] = cmat[6]; }
  normalize3(d);
  double e[3];
  cross3(e, ax, d);
  /* the deeper cap: the one whose centre is lower along the normal */
  double sdeep = an > 0 ? -1.0 : 1.0;
  for (int cap = 0; cap < 2; ++cap) {
    double sc = cap == 0 ? sdeep : -sdeep;
    int npts = cap == 0 ? 3 : 1;
    for (int k = 0; k < npts; ++k) {
      double cu = k == 0 ? 1.0 : -0.5, cv = k == 0 ? 0.0 : (k == 1 ? 0.8660254037844386 : -0.8660254037844386);
      double p[3], dv[3];
      for (int i = 0; i < 3; ++i) p[i] = cpos[i] + sc * size[1] * ax[i] + size[0] * (cu * d[i] + cv * e[i]);
      for (int i = 0; i < 3; ++i) dv[i] = p[i] - ppos[i];
      double dist = dot3(dv, nrm);
      if (dist > margin) continue;
      double pos[3];
      for (int i = 0; i < 3; ++i) pos[i] = p[i] - nrm[i] * dist / 2;
      n = add_contact(out, n, dist, pos, nrm);
    }
  }
  return n;
}
/* plane vs mesh: every convex-hull vertex within margin, in hull order (at most 8) */
static int col_plane_mesh(const mrs_model_view* m, orc_ws* w, const double* ppos, const double* pmat, int g2,
                          double margin, orc_contact* out, int n) {
  orc_shape B;
  shape_of(m, w, g2, 0, &B);
  double nrm[3] = {pmat[2], pmat[5], pmat[8]};
  for (int k = 0; k < B.nhull; ++k) {
    double p[3], dv[3];
    mat_vec(p, B.mat, B.vert + 3 * B.hull[k]);
    for (int i = 0; i < 3; ++i) { p[i] += B.pos[i]; dv[i] = p[i] - ppos[i]; }
    double dist = dot3(dv, nrm);
    if (dist > margin) continue;
    double pos[3];
    for (int i = 0; i < 3; ++i) pos[i] = p[i] - nrm[i] * dist / 2;
    n = add_contact(out, n, dist, pos, nrm);
  }
  return n;
}

static int narrowphase(const mrs_model_view* m, orc_ws* w, int g1, int g2, double margin, orc_contact* out) {
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const double *p1 = w->geom_xpos + 3 * g1, *p2 = w->geom_xpos + 3 * g2;
  const double *m1 = w->geom_xmat + 9 * g1, *m2 = w->geom_xmat + 9 * g2;
  const double *s1 = m->geom_size + 3 * g1, *s2 = m->geom_size + 3 * g2;
  double a1[3], b1[3], a2[3], b2[3], c1[3], c2[3];
  int n = 0;
  if (t1 == MRS_GEOM_PLANE) {
    switch (t2) {
      case MRS_GEOM_SPHERE: return col_plane_sphere(p1, m1, p2, s2[0], margin, out, 0);
      case MRS_GEOM_CAPSULE:
        capsule_ends(p2, m2, s2[1], a2, b2);
        n = col_plane_sphere(p1, m1, a2, s2[0], margin, out, 0);
        return col_plane_sphere(p1, m1, b2, s2[0], margin, out, n);
      case MRS_GEOM_BOX: return col_plane_box(p1, m1, p2, m2, s2, margin, out, 0);
      case MRS_GEOM_ELLIPSOID: return col_plane_convex_support(m, w, p1, m1, g2, margin, out, 0);
      case MRS_GEOM_CYLINDER: return col_plane_cylinder(p1, m1, p2, m2, s2, margin, out, 0);
      case MRS_GEOM_MESH: return col_plane_mesh(m, w, p1, m1, g2, margin, out, 0);
    }
    return -1;
  } else if (t1 == MRS_GEOM_SPHERE) {
    switch (t2) {
      case MRS_GEOM_SPHERE: return col_sphere_sphere(p1, s1[0], p2, s2[0], margin, out, 0);
      case MRS_GEOM_CAPSULE:
        capsule_ends(p2, m2, s2[1], a2, b2);
        segment_point_closest(a2, b2, p1, c2);
        return col_sphere_sphere(p1, s1[0], c2, s2[0], margin, out, 0);
      case MRS_GEOM_BOX: return col_sphere_box(p1, s1[0], p2, m2, s2, margin, out, 0);
    }
  } else if (t1 == MRS_GEOM_CAPSULE) {
    switch (t2) {
      case MRS_GEOM_CAPSULE:
        capsule_ends(p1, m1, s1[1], a1, b1);
        capsule_ends(p2, m2, s2[1], a2, b2);
        segment_segment_closest(a1, b1, a2, b2, c1, c2);
        return col_sphere_sphere(c1, s1[0], c2, s2[0], margin, out, 0);
      case MRS_GEOM_BOX:
        capsule_ends(p1, m1, s1[1], a1, b1);
        return col_capsule_box(a1, b1, s1[0], p2, m2, s2, margin, out, 0);
    }
  } else if (t1 == MRS_GEOM_BOX && t2 == MRS_GEOM_BOX) {
    return col_box_box(p1, m1, s1, p2, m2, s2, margin, out, 0);
  }
  /* every other pair has an ellipsoid, cylinder or mesh: general convex (MPR) */
  if (t1 != MRS_GEOM_HFIELD && t2 != MRS_GEOM_HFIELD) return col_convex(m, w, g1, g2, margin, out, 0);
  return -1; /* unsupported pair */
}

/* static broad-phase filters of mj_collision [upstream mj_collideGeoms / filterBitmask]: different
 * weld groups, not parent-child welds (world never filtered), contype/conaffinity compatible */
static int pair_admissible(const mrs_model_view* m, int g1, int g2) {
  int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
  int w1 = m->body_weldid[b1], w2 = m->body_weldid[b2];
  if (w1 == w2) return 0;
  if (!(m->disableflags & MRS_DSBL_FILTERPARENT) && w1 != 0 && w2 != 0 &&
      (w1 == m->body_weldid[m->body_parentid[w2]] || w2 == m->body_weldid[m->body_parentid[w1]]))
    return 0;
  if (!((m->geom_contype[g1] & m->geom_conaffinity[g2]) || (m->geom_contype[g2] & m->geom_conaffinity[g1])))
    return 0;
  /* body pairs excluded by <contact><exclude> (exclude signatures), or the very geom pair an explicit
   * <pair> names: mj_collision's merge skips, among a body pair's dynamic geom pairs, only those in the
   * explicit list of the same body signature; the bodies' other geoms still collide dynamically
   * [upstream engine_collision_driver.c mj_collideGeoms merge test; verify] */
  const int lo = b1 < b2 ? b1 : b2, hi = b1 < b2 ? b2 : b1;
  for (int k = 0; k < m->nexclude; ++k)
    if (m->exclude_body1[k] == lo && m->exclude_body2[k] == hi) return 0;
  for (int k = 0; k < m->nexpair; ++k) {
    const int e1 = m->expair_geom1[k], e2 = m->expair_geom2[k];
    if ((e1 == g1 && e2 == g2) || (e1 == g2 && e2 == g1)) return 0;
  }
  return 1;
}

int orc_candidate_pairs(const mrs_model_view* m, int max, int* geom1, int* geom2) {
  int n = 0;
  if (m->disableflags & (MRS_DSBL_CONTACT | MRS_DSBL_CONSTRAINT)) return 0;
  for (int g1 = 0; g1 < m->ngeom; ++g1)
    for (int g2 = g1 + 1; g2 < m->ngeom; ++g2) {
      if (!pair_admissible(m, g1, g2)) continue;
      if (n < max) {
        int swap = m->geom_type[g1] > m->geom_type[g2];
        geom1[n] = swap ? g2 : g1;
        geom2[n] = swap ? g1 : g2;
      }
      ++n;
    }
  return n;
}

static void collision(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  w->ncon = 0;
  if (m->disableflags & (MRS_DSBL_CONTACT | MRS_DSBL_CONSTRAINT)) return;
  /* explicit <contact><pair>s first, with their own parameters (geom1 has the lower type) */
  for (int k = 0; k < m->nexpair; ++k) {
    const int ga = m->expair_geom1[k], gb = m->expair_geom2[k];
    const double margin = m->expair_margin[k], gap = m->expair_gap[k];
    if (m->geom_type[ga] != MRS_GEOM_PLANE && m->geom_type[gb] != MRS_GEOM_PLANE) {
      double dv[3];
      for (int i = 0; i < 3; ++i) dv[i] = w->geom_xpos[3 * ga + i] - w->geom_xpos[3 * gb + i];
      if (norm3(dv) > m->geom_rbound[ga] + m->geom_rbound[gb] + margin) continue;
    }
    orc_contact tmp[8];
    const int nc = narrowphase(m, w, ga, gb, margin, tmp);
    for (int c = 0; c < nc && w->ncon < MAXCON; ++c) {
      orc_contact* o = &w->con[w->ncon++];
      *o = tmp[c];
      o->geom[0] = ga; o->geom[1] = gb;
      o->dim = m->expair_dim[k];
      o->friction[0] = m->expair_friction[5 * k];
      o->friction[1] = m->expair_friction[5 * k + 2];
      o->friction[2] = m->expair_friction[5 * k + 3];
      for (int i = 0; i < 2; ++i) o->solref[i] = m->expair_solref[2 * k + i];
      for (int i = 0; i < 5; ++i) o->solimp[i] = m->expair_solimp[5 * k + i];
      o->includemargin = margin - gap;
    }
  }
  for (int g1 = 0; g1 < m->ngeom; ++g1)
    for (int g2 = g1 + 1; g2 < m->ngeom; ++g2) {
      if (!pair_admissible(m, g1, g2)) continue;
      double margin = fmax(m->geom_margin[g1], m->geom_margin[g2]);
      double gap = fmax(m->geom_gap[g1], m->geom_gap[g2]);
      if (m->geom_type[g1] != MRS_GEOM_PLANE && m->geom_type[g2] != MRS_GEOM_PLANE) {
        double dv[3];
        for (int i = 0; i < 3; ++i) dv[i] = w->geom_xpos[3 * g1 + i] - w->geom_xpos[3 * g2 + i];
        if (norm3(dv) > m->geom_rbound[g1] + m->geom_rbound[g2] + margin) continue;
      }
      int ga = g1, gb = g2;
      if (m->geom_type[ga] > m->geom_type[gb]) { ga = g2; gb = g1; }
      orc_contact tmp[8]; /* a pair gives at most 8 contacts (box-box face polygon) */
      int nc = narrowphase(m, w, ga, gb, margin, tmp);
      if (nc < 0) continue; /* unsupported pairs are rejected at batch creation in the product */
      /* contact parameters [upstream mj_contactParam]: max friction/condim, solmix-weighted solref */
      double mix, s1 = m->geom_solmix[ga], s2 = m->geom_solmix[gb];
      if (s1 >= MINVAL && s2 >= MINVAL) mix = s1 / (s1 + s2);
      else if (s1 < MINVAL && s2 < MINVAL) mix = 0.5;
      else mix = s1 < MINVAL ? 0 : 1;
      for (int k = 0; k < nc && w->ncon < MAXCON; ++k) {
        orc_contact* c = &w->con[w->ncon++];
        *c = tmp[k];
        c->geom[0] = ga; c->geom[1] = gb;
        c->dim = m->geom_condim[ga] > m->geom_condim[gb] ? m->geom_condim[ga] : m->geom_condim[gb];
        for (int i = 0; i < 3; ++i) c->friction[i] = fmax(m->geom_friction[3 * ga + i], m->geom_friction[3 * gb + i]);
        for (int i = 0; i < 2; ++i) c->solref[i] = mix * m->geom_solref[2 * ga + i] + (1 - mix) * m->geom_solref[2 * gb + i];
        for (int i = 0; i < 5; ++i) c->solimp[i] = mix * m->geom_solimp[5 * ga + i] + (1 - mix) * m->geom_solimp[5 * gb + i];
        c->includemargin = margin - gap;
      }
    }
}

/* ------------------------------------------------------------------------ constraints
 * mj_makeConstraint [upstream engine_core_constraint.c]: dof friction loss rows, joint limit rows
 * (lower then upper, active when dist < margin), pyramidal contact rows (condim 3: four edges
 * J_n +/- mu_k J_tk).  mj_makeImpedance: impedance from solimp, R = (1-imp)/imp * diagApprox,
 * aref = -B v - K imp (pos - margin). */
static double impedance(const double* solimp, double pos, double margin) {
  double dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  dmin = dmin < 0.0001 ? 0.0001 : dmin > 0.9999 ? 0.9999 : dmin;
  dmax = dmax < 0.0001 ? 0.0001 : dmax > 0.9999 ? 0.9999 : dmax;
  if (dmin == dmax || width <= MINVAL) return 0.5 * (dmin + dmax);
  double x = fabs(pos - margin) / width;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  double y;
  if (power == 1) y = x;
  else if (x <= mid) y = pow(x, power) / pow(mid, power - 1);
  else y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
  return dmin + y * (dmax - dmin);
}

static void add_row(orc_ws* w, int nv, int type, int id, const double* J, double pos, double margin,
                    double floss, double diag, const double* solref, const double* solimp) {
  if (w->nefc >= MAXEFC) return;
  int r = w->nefc++;
  memcpy(w->efc_J + (size_t)r * nv, J, nv * sizeof(double));
  w->efc_type[r] = type; w->efc_id[r] = id;
  w->efc_pos[r] = pos; w->efc_margin[r] = margin; w->efc_frictionloss[r] = floss;
  w->efc_diag[r] = diag;
  w->efc_rscale[r] = 1;
  w->efc_sub[r] = -1;
  memcpy(w->efc_solref[r], solref, 2 * sizeof(double));
  memcpy(w->efc_solimp[r], solimp, 5 * sizeof(double));
}

/* equality rows [upstream mj_instantiateEquality; restated, verify], first as mj_makeConstraint
 * orders them (eq_data layout: include/mrs_model.h):
 *   connect: p1 - p2 of the anchor on body1 and its qpos0 image on body2, 3 rows, J = J_p1 - J_p2,
 *            diagApprox the bodies' translational invweight0;
 *   weld:    the same for body2's anchor and where body1's relpose puts it (3 rows), then the rotation
 *            error imag(e) * torquescale, e = conj(q1 relquat) q2 (3 rows; J column = the exact
 *            derivative 1/2 imag(conj(q1 relquat) (w2 - w1) q2) of that error for the dof's angular
 *            motion), diagApprox rotational invweight0;
 *   joint:   (q1 - q1_0) - poly(q2 - q2_0), J = e_dof1 - poly'(q2 - q2_0) e_dof2, diagApprox the
 *            dofs' invweight0.
 * Unbounded (EQ_BOUND), position term as limits. */
static void equality_rows(const mrs_model_view* m, orc_data* d, orc_ws* w, double* J) {
  const int nv = m->nv;
  for (int q = 0; q < m->neq; ++q) {
    if (!m->eq_active0[q]) continue;
    const double* dd = m->eq_data + MRS_NEQDATA * q;
    const double* sr = m->eq_solref + 2 * q;
    const double* si = m->eq_solimp + 5 * q;
    const int t = m->eq_type[q], o1 = m->eq_obj1id[q], o2 = m->eq_obj2id[q];
    if (t == MRS_EQ_JOINT) {
      const int d1 = m->jnt_dofadr[o1];
      const double x1 = d->qpos[m->jnt_qposadr[o1]] - dd[5];
      double poly = dd[0], dpoly = 0, diag = m->dof_invweight0[d1];
      memset(J, 0, nv * sizeof(double));
      J[d1] = 1;
      if (o2 >= 0) {
        const int d2 = m->jnt_dofadr[o2];
        const double x = d->qpos[m->jnt_qposadr[o2]] - dd[6];
        poly = dd[0] + x * (dd[1] + x * (dd[2] + x * (dd[3] + x * dd[4])));
        dpoly = dd[1] + x * (2 * dd[2] + x * (3 * dd[3] + x * 4 * dd[4]));
        J[d2] -= dpoly;
        diag += m->dof_invweight0[d2];
      }
      add_row(w, nv, EFC_EQUALITY, q, J, x1 - poly, 0, EQ_BOUND, diag, sr, si);
      continue;
    }
    /* anchor points on body1 (p1) and body2 (p2) */
    const double *q1 = w->xquat + 4 * o1, *q2 = w->xquat + 4 * o2;
    double l1[3], l2[3], p1[3], p2[3], r[3], q1r[4];
    if (t == MRS_EQ_CONNECT) {
      for (int i = 0; i < 3; ++i) { l1[i] = dd[i]; l2[i] = dd[3 + i]; }
    } else {
      double ra[3];
      double m6[9];
      quat2mat(m6, dd + 6);
      mat_vec(ra, m6, dd);
      for (int i = 0; i < 3; ++i) { l2[i] = dd[i]; l1[i] = dd[3 + i] + ra[i]; }
    }
    mat_vec(r, w->xmat + 9 * o1, l1);
    for (int i = 0; i < 3; ++i) p1[i] = w->xpos[3 * o1 + i] + r[i];
    mat_vec(r, w->xmat + 9 * o2, l2);
    for (int i = 0; i < 3; ++i) p2[i] = w->xpos[3 * o2 + i] + r[i];
    const double tdiag = m->body_invweight0[2 * o1] + m->body_invweight0[2 * o2];
    for (int k = 0; k < 3; ++k) {
      for (int j = 0; j < nv; ++j) {
        double c1[3] = {0, 0, 0}, c2[3] = {0, 0, 0};
        if (dof_affects(m, j, o1)) jac_point_col(m, w, o1, p1, j, c1);
        if (dof_affects(m, j, o2)) jac_point_col(m, w, o2, p2, j, c2);
        J[j] = c1[k] - c2[k];
      }
      add_row(w, nv, EFC_EQUALITY, q, J, p1[k] - p2[k], 0, EQ_BOUND, tdiag, sr, si);
    }
    if (t != MRS_EQ_WELD) continue;
    const double ts = dd[10];
    double cq[4], e[4], tmp[4];
    quat_mul(q1r, q1, dd + 6);
    cq[0] = q1r[0]; cq[1] = -q1r[1]; cq[2] = -q1r[2]; cq[3] = -q1r[3];
    quat_mul(e, cq, q2);
    const double rdiag = m->body_invweight0[2 * o1 + 1] + m->body_invweight0[2 * o2 + 1];
    for (int k = 0; k < 3; ++k) {
      for (int j = 0; j < nv; ++j) {
        double wv[4] = {0, 0, 0, 0};
        for (int i = 0; i < 3; ++i) {
          if (dof_affects(m, j, o2)) wv[1 + i] += w->cdof[6 * j + i];
          if (dof_affects(m, j, o1)) wv[1 + i] -= w->cdof[6 * j + i];
        }
        quat_mul(tmp, cq, wv);
        double de[4];
        quat_mul(de, tmp, q2);
        J[j] = 0.5 * de[1 + k] * ts;
      }
      add_row(w, nv, EFC_EQUALITY, q, J, e[1 + k] * ts, 0, EQ_BOUND, rdiag, sr, si);
    }
  }
}

static void make_constraint(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  int nv = m->nv;
  w->nefc = 0;
  if (m->disableflags & MRS_DSBL_CONSTRAINT) return;
  double* J = (double*)malloc(nv * sizeof(double) + 8);
  if (!(m->disableflags & MRS_DSBL_EQUALITY)) equality_rows(m, d, w, J);
  if (!(m->disableflags & MRS_DSBL_FRICTIONLOSS))
    for (int j = 0; j < nv; ++j) {
      if (m->dof_frictionloss[j] <= 0) continue;
      memset(J, 0, nv * sizeof(double));
      J[j] = 1;
      add_row(w, nv, EFC_FRICTION, j, J, 0, 0, m->dof_frictionloss[j], m->dof_invweight0[j],
              m->dof_solref + 2 * j, m->dof_solimp + 5 * j);
    }
  /* tendon friction loss rows [upstream mj_instantiateFriction: after the dofs'], J = ten_J */
  if (!(m->disableflags & MRS_DSBL_FRICTIONLOSS))
    for (int t = 0; t < m->ntendon; ++t) {
      if (m->tendon_frictionloss[t] <= 0) continue;
      tendon_length(m, d, t, J, NULL);
      add_row(w, nv, EFC_TFRICTION, t, J, 0, 0, m->tendon_frictionloss[t], m->tendon_invweight0[t],
              m->tendon_solref_fri + 2 * t, m->tendon_solimp_fri + 5 * t);
    }
  if (!(m->disableflags & MRS_DSBL_LIMIT))
    for (int j = 0; j < m->njnt; ++j) {
      if (!m->jnt_limited[j]) continue;
      int t = m->jnt_type[j];
      if (t != MRS_JNT_HINGE && t != MRS_JNT_SLIDE) continue;
      double q = d->qpos[m->jnt_qposadr[j]], margin = m->jnt_margin[j];
      int da = m->jnt_dofadr[j];
      for (int side = -1; side <= 1; side += 2) {
        double dist = side * (m->jnt_range[2 * j + (side + 1) / 2] - q);
        if (dist < margin) {
          memset(J, 0, nv * sizeof(double));
          J[da] = -side;
          add_row(w, nv, EFC_LIMIT, j, J, dist, margin, 0, m->dof_invweight0[da],
                  m->jnt_solref + 2 * j, m->jnt_solimp + 5 * j);
        }
      }
    }
  /* tendon limit rows [upstream mj_instantiateLimit: after the joints'], lower then upper, J = +-ten_J */
  if (!(m->disableflags & MRS_DSBL_LIMIT))
    for (int t = 0; t < m->ntendon; ++t) {
      if (!m->tendon_limited[t]) continue;
      const double L = tendon_length(m, d, t, J, NULL), margin = m->tendon_margin[t];
      for (int side = -1; side <= 1; side += 2) {
        const double dist = side * (m->tendon_range[2 * t + (side + 1) / 2] - L);
        if (dist < margin) {
          double* Js = (double*)malloc(nv * sizeof(double) + 8);
          for (int i = 0; i < nv; ++i) Js[i] = -side * J[i];
          add_row(w, nv, EFC_TLIMIT, t, Js, dist, margin, 0, m->tendon_invweight0[t],
                  m->tendon_solref_lim + 2 * t, m->tendon_solimp_lim + 5 * t);
          free(Js);
        }
      }
    }
  /* contacts */
  for (int c = 0; c < w->ncon; ++c) {
    orc_contact* con = &w->con[c];
    int b1 = m->geom_bodyid[con->geom[0]], b2 = m->geom_bodyid[con->geom[1]];
    double tran = m->body_invweight0[2 * b1] + m->body_invweight0[2 * b2];
    double* Jc = (double*)calloc(3 * (size_t)nv, sizeof(double)); /* rows: normal, t1, t2 */
    for (int j = 0; j < nv; ++j) {
      double col1[3] = {0, 0, 0}, col2[3] = {0, 0, 0};
      if (dof_affects(m, j, b1)) jac_point_col(m, w, b1, con->pos, j, col1);
      if (dof_affects(m, j, b2)) jac_point_col(m, w, b2, con->pos, j, col2);
      double dc[3] = {col2[0] - col1[0], col2[1] - col1[1], col2[2] - col1[2]};
      for (int r = 0; r < 3; ++r) Jc[r * nv + j] = dot3(con->frame + 3 * r, dc);
    }
    w->efc_con_first[c] = w->nefc;
    if (con->dim == 3 && m->cone == MRS_CONE_ELLIPTIC) {
      /* elliptic cone [upstream mj_instantiateContact / mj_makeImpedance, restated; verify]: rows J_n,
       * J_t1, J_t2 of the contact frame, diagApprox tran for each; the impedance of the normal for all
       * three; the tangents' regulariser R_n mu_1^2 / (mu_j^2 impratio) = R_n / impratio (both tangents
       * use the sliding coefficient); the cone's regularised mu = mu_1 / sqrt(impratio) */
      if (w->nefc + 3 <= MAXEFC)
        for (int k = 0; k < 3; ++k) {
          add_row(w, nv, EFC_CONTACT, c, Jc + (size_t)k * nv, con->dist, con->includemargin, 0, tran, con->solref,
                  con->solimp);
          w->efc_sub[w->nefc - 1] = k;
          w->efc_rscale[w->nefc - 1] = k == 0 ? 1 : 1 / m->impratio;
          w->efc_fr[w->nefc - 1] = con->friction[0];
          w->efc_mu[w->nefc - 1] = con->friction[0] / sqrt(m->impratio);
        }
    } else if (con->dim == 1) {
      add_row(w, nv, EFC_CONTACT, c, Jc, con->dist, con->includemargin, 0, tran, con->solref, con->solimp);
    } else {
      /* pyramid edges J_n +/- mu J_tk.  diagApprox of an edge is tran (1 + mu^2) [upstream
       * mj_diagApprox]; mj_makeImpedance then gives every edge of the pyramid the regulariser
       * R_py = 2 mu^2 R / impratio, which matches the elliptic cone's frictional regulariser
       * R_t = R_n / impratio on the tangent components (two edges per direction, each carrying half
       * the normal load): rscale below */
      const double mu = con->friction[0];
      for (int k = 1; k < 3; ++k)
        for (int s = 1; s >= -1; s -= 2) {
          /* both tangent directions use the sliding coefficient: a contact's friction is
           * (slide, slide, spin, roll, roll) from the geoms' (slide, spin, roll) [upstream mj_setContact] */
          for (int j = 0; j < nv; ++j) J[j] = Jc[j] + s * mu * Jc[k * nv + j];
          add_row(w, nv, EFC_CONTACT, c, J, con->dist, con->includemargin, 0,
                  tran * (1 + mu * mu), con->solref, con->solimp);
          if (w->nefc > 0) w->efc_rscale[w->nefc - 1] = 2 * mu * mu / m->impratio;
        }
    }
    free(Jc);
  }
  free(J);
  /* impedance, R, D, aref */
  for (int r = 0; r < w->nefc; ++r) {
    const double* sr = w->efc_solref[r];
    double imp = impedance(w->efc_solimp[r], w->efc_pos[r], w->efc_margin[r]);
    double R = (1 - imp) * w->efc_diag[r] * w->efc_rscale[r] / imp;
    w->efc_R[r] = R > MINVAL ? R : MINVAL;
    w->efc_D[r] = 1 / w->efc_R[r];
    double K, B;
    double dmax = w->efc_solimp[r][1];
    dmax = dmax < 0.0001 ? 0.0001 : dmax > 0.9999 ? 0.9999 : dmax;
    if (sr[0] > 0) {
      double tc = sr[0], dr = sr[1];
      if (!(m->disableflags & MRS_DSBL_REFSAFE) && tc < 2 * m->timestep) tc = 2 * m->timestep;
      K = 1 / (dmax * dmax * tc * tc * dr * dr);
      B = 2 / (dmax * tc);
    } else {
      K = -sr[0] / (dmax * dmax);
      B = -sr[1] / dmax;
    }
    double vel = 0;
    for (int j = 0; j < nv; ++j) vel += w->efc_J[(size_t)r * nv + j] * d->qvel[j];
    w->efc_vel[r] = vel;
    /* (friction loss rows and the tangent rows of an elliptic cone carry no position term) */
    double pterm = (w->efc_type[r] == EFC_FRICTION || w->efc_type[r] == EFC_TFRICTION || w->efc_sub[r] > 0)
                       ? 0 : K * imp * (w->efc_pos[r] - w->efc_margin[r]);
    w->efc_aref[r] = -B * vel - pterm;
    w->efc_KBIP[r][0] = K; w->efc_KBIP[r][1] = B; w->efc_KBIP[r][2] = imp; w->efc_KBIP[r][3] = 0;
  }
}

/* ---- elliptic cones [upstream mj_constraintUpdate elliptic branch, restated; verify].  In the
 * regularised cone space U = (mu jar_n, mu_t jar_t1, mu_t jar_t2) (mu = the block's efc_mu, mu_t = its
 * friction coefficient), N = U_0, T = |U_t|:
 *   top zone    N >= mu T:         no force, no cost;
 *   bottom zone mu N + T <= 0:     every row quadratic, f_j = -D_j jar_j, cost 1/2 sum D_j jar_j^2;
 *   middle zone otherwise:         cost 1/2 Dm (N - mu T)^2 with Dm = D_n / (mu^2 (1 + mu^2)),
 *                                  f = -d cost / d jar, Hessian S H_U S (S = diag(mu, mu_t, mu_t)),
 *                                  H_U = Dm [[1, -mu U_t'/T], [-mu U_t/T, mu N/T^3 U_t U_t' + (mu^2 - mu N/T) I]].
 * Returns the zone as a row state (ST_SAT, ST_QUAD, ST_CONE); f, cost and H (3x3, jar space) may be
 * NULL. */
enum { ST_CONE = 4 };
static int ell_block(const orc_ws* w, int r, const double jar[3], double f[3], double* cost, double H[9]) {
  const double mu = w->efc_mu[r], ft = w->efc_fr[r];
  const double U[3] = {mu * jar[0], ft * jar[1], ft * jar[2]};
  const double N = U[0], T = sqrt(U[1] * U[1] + U[2] * U[2]);
  if (N >= mu * T || (T <= 0 && N >= 0)) {
    if (f) f[0] = f[1] = f[2] = 0;
    if (cost) *cost = 0;
    if (H) memset(H, 0, 9 * sizeof(double));
    return 0; /* ST_SAT */
  }
  if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
    double c = 0;
    for (int j = 0; j < 3; ++j) {
      if (f) f[j] = -w->efc_D[r + j] * jar[j];
      c += 0.5 * w->efc_D[r + j] * jar[j] * jar[j];
    }
    if (cost) *cost = c;
    if (H) {
      memset(H, 0, 9 * sizeof(double));
      for (int j = 0; j < 3; ++j) H[4 * j] = w->efc_D[r + j];
    }
    return 1; /* ST_QUAD */
  }
  const double Dm = w->efc_D[r] / (mu * mu * (1 + mu * mu)), NT = N - mu * T;
  if (cost) *cost = 0.5 * Dm * NT * NT;
  if (f) {
    f[0] = -Dm * NT * mu;
    for (int j = 1; j < 3; ++j) f[j] = Dm * NT * mu / T * U[j] * ft;
  }
  if (H) {
    const double S[3] = {mu, ft, ft};
    double HU[9];
    HU[0] = 1;
    for (int j = 1; j < 3; ++j) HU[j] = HU[3 * j] = -mu * U[j] / T;
    for (int j = 1; j < 3; ++j)
      for (int k = 1; k < 3; ++k)
        HU[3 * j + k] = mu * N / (T * T * T) * U[j] * U[k] + (j == k ? mu * mu - mu * N / T : 0);
    for (int j = 0; j < 3; ++j)
      for (int k = 0; k < 3; ++k) H[3 * j + k] = Dm * S[j] * HU[3 * j + k] * S[k];
  }
  return ST_CONE;
}

/* mju_QCQP2 [upstream engine_util_solve.c, restated]: min 1/2 x'Ax + x'b s.t. sum (x_i / d_i)^2 <= r^2
 * over 2 variables: scaled to the unit-coefficient ball, Newton on the multiplier la of the active
 * constraint (A + la I) y = -b, |y| = r, at most 20 iterations, stopping when |y|^2 - r^2 < 1e-10 or the
 * step < 1e-10; returns 1 when the constraint is active */
static double qcqp2_la(double res[2], const double A[4], const double b[2], const double d[2], double r);
static int qcqp2(double res[2], const double A[4], const double b[2], const double d[2], double r) {
  return qcqp2_la(res, A, b, d, r) != 0;
}
/* ... and its multiplier: la of (A_s + la I) y = -b_s in the scaled variables y = x / d */
static double qcqp2_la(double res[2], const double A[4], const double b[2], const double d[2], double r) {
  const double b1 = b[0] * d[0], b2 = b[1] * d[1];
  const double A11 = A[0] * d[0] * d[0], A22 = A[3] * d[1] * d[1], A12 = A[1] * d[0] * d[1];
  double la = 0, v1 = 0, v2 = 0;
  for (int it = 0; it < 20; ++it) {
    const double det = (A11 + la) * (A22 + la) - A12 * A12;
    if (det < 1e-10) { res[0] = res[1] = 0; return 0; }
    const double di = 1 / det, P11 = (A22 + la) * di, P22 = (A11 + la) * di, P12 = -A12 * di;
    v1 = -P11 * b1 - P12 * b2;
    v2 = -P12 * b1 - P22 * b2;
    const double val = v1 * v1 + v2 * v2 - r * r;
    if (val < 1e-10) break;
    const double deriv = -2.0 * (P11 * v1 * v1 + 2.0 * P12 * v1 * v2 + P22 * v2 * v2);
    const double delta = -val / deriv;
    if (delta < 1e-10) break;
    la += delta;
  }
  res[0] = v1 * d[0];
  res[1] = v2 * d[1];
  return la;
}

/* the exact minimiser of 1/2 y'Ay + y'c over the elliptic cone K = {|y_t| <= mu y_n} (3x3 block):
 * g(s) = min over |x| <= mu s of the block cost at y = (s, x) (mju_QCQP2) is convex in s, with
 * g'(s) = (A y + c)_n - la s (envelope theorem; la the QCQP's multiplier), so s is found by a safeguarded
 * secant / bisection on g' over s >= 0 (s = 0, i.e. y = 0, when g'(0+) = c_n - mu |c_t| >= 0). */
static void ell_block_min(const double A[9], const double c[3], double mu, double y[3]) {
  const double At[4] = {A[4], A[5], A[7], A[8]}, dd[2] = {mu, mu};
  /* y(s) and g'(s) */
  double x[2];
  /* g'(0+) = c_n - mu |c_t| (the friction takes the boundary at once): the apex y = 0 is optimal
   * when c lies in the dual cone */
  double gp_lo = c[0] - mu * sqrt(c[1] * c[1] + c[2] * c[2]), s_lo = 0, s_hi, gp_hi;
  if (gp_lo >= 0) { y[0] = y[1] = y[2] = 0; return; }
  #define ELL_EVAL(S, GP)                                                                  \
    do {                                                                                   \
      const double s_ = (S);                                                               \
      const double bc_[2] = {c[1] + A[3] * s_, c[2] + A[6] * s_};                          \
      const double la_ = qcqp2_la(x, At, bc_, dd, s_);                                     \
      (GP) = A[0] * s_ + A[1] * x[0] + A[2] * x[1] + c[0] - la_ * s_;                      \
    } while (0)
  s_hi = -c[0] / A[0];
  if (s_hi <= 0) s_hi = 1;
  for (int k = 0; k < 60; ++k) {
    ELL_EVAL(s_hi, gp_hi);
    if (gp_hi >= 0) break;
    s_lo = s_hi; gp_lo = gp_hi;
    s_hi *= 2;
  }
  double s_ = s_hi;
  for (int it = 0; it < 100 && s_hi - s_lo > 1e-14 * (1 + s_hi); ++it) {
    /* secant step inside the bracket, bisection when it stalls near an end */
    double sn = s_lo - gp_lo * (s_hi - s_lo) / (gp_hi - gp_lo);
    if (!(sn > s_lo + 0.01 * (s_hi - s_lo) && sn < s_hi - 0.01 * (s_hi - s_lo))) sn = 0.5 * (s_lo + s_hi);
    double gp;
    ELL_EVAL(sn, gp);
    s_ = sn;
    if (gp == 0) { s_lo = s_hi = sn; break; }
    if (gp < 0) { s_lo = sn; gp_lo = gp; } else { s_hi = sn; gp_hi = gp; }
  }
  #undef ELL_EVAL
  s_ = 0.5 * (s_lo + s_hi);
  const double bc[2] = {c[1] + A[3] * s_, c[2] + A[6] * s_};
  qcqp2_la(x, At, bc, dd, s_);
  y[0] = s_; y[1] = x[0]; y[2] = x[1];
}

/* mj_solPGS's update of one elliptic contact block [upstream engine_solver.c; restated from the
 * published engine, verify]: with res = AR f + b at the old forces f_old and A the block of AR,
 *   1. normal or ray step: when the old normal force is 0, the normal's own 1-D step
 *      f_n -= res_n / A_nn, clamped at 0; otherwise the exact minimiser along the ray of the old force
 *      v = f_old, x = -(v'res) / (v'A v), shortened so the normal stays >= 0;
 *   2. friction with the normal fixed: min over f_t of the block cost, |f_t| <= mu f_n, by mju_QCQP2
 *      (zero friction when f_n is 0).
 * A block whose normal diagonal is below MINVAL keeps its forces. */
static void ell_pgs_split(const double A[9], const double res[3], const double old[3], double mu, double y[3]) {
  y[0] = old[0]; y[1] = old[1]; y[2] = old[2];
  if (A[0] < MINVAL) return;
  if (old[0] < MINVAL) {
    y[0] = old[0] - res[0] / A[0];
    if (y[0] < 0) y[0] = 0;
  } else {
    double Av[3], vAv = 0, vr = 0;
    for (int k = 0; k < 3; ++k) Av[k] = A[3 * k] * old[0] + A[3 * k + 1] * old[1] + A[3 * k + 2] * old[2];
    for (int k = 0; k < 3; ++k) { vAv += old[k] * Av[k]; vr += old[k] * res[k]; }
    if (vAv >= MINVAL) {
      double x = -vr / vAv;
      if (old[0] + x * old[0] < 0) x = -1;
      for (int k = 0; k < 3; ++k) y[k] = old[k] + x * old[k];
    }
  }
  if (y[0] < MINVAL) { y[0] = y[0] < 0 ? 0 : y[0]; y[1] = y[2] = 0; return; }
  /* friction: 1/2 x'A_tt x + x'(res_t + A_tn (y_n - f_old,n) - A_tt f_old,t) over |x| <= mu y_n */
  const double At[4] = {A[4], A[5], A[7], A[8]}, dd[2] = {mu, mu};
  const double dn = y[0] - old[0];
  const double bt[2] = {res[1] + A[3] * dn - (A[4] * old[1] + A[5] * old[2]),
                        res[2] + A[6] * dn - (A[7] * old[1] + A[8] * old[2])};
  double x[2];
  qcqp2(x, At, bt, dd, y[0]);
  y[1] = x[0]; y[2] = x[1];
}

/* force of one row for a given jar = J qacc - aref (mj_constraintUpdate primal states) */
static double row_force(orc_ws* w, int r, double jar) {
  double D = w->efc_D[r];
  if (FRIC_LIKE(w->efc_type[r])) {
    double fl = w->efc_frictionloss[r], Rr = w->efc_R[r];
    if (jar <= -Rr * fl) return fl;
    if (jar >= Rr * fl) return -fl;
    return -D * jar;
  }
  return jar < 0 ? -D * jar : 0;
}

/* ---- primal solvers: mj_solNewton / mj_solCG [upstream engine_solver.c, mj_solPrimal].
 * Both minimise over qacc the convex cost
 *   F(qacc) = 1/2 (qacc - qacc_smooth)' M (qacc - qacc_smooth) + sum_r s_r(J_r qacc - aref_r)
 * with the soft-constraint row costs of mj_constraintUpdate (s_r on jar = J_r qacc - aref_r):
 *   limit / contact rows: 1/2 D jar^2 when jar < 0, else 0;
 *   friction-loss rows:   1/2 D jar^2 inside |jar| < R floss, linear floss |jar| - 1/2 R floss^2 outside.
 * Newton: search = -H^-1 grad with H = M + J' diag(D of quadratic rows) J (mj_solNewton's Hessian;
 * upstream updates its factor incrementally, the matrix is the same); CG: Polak-Ribiere with the
 * M^-1 preconditioner.  Exact line search along the search direction: safeguarded 1-D Newton on
 * the piecewise-quadratic F(qacc + a p) (upstream PrimalLinesearch brackets with Newton steps to
 * |dF/da| < tolerance * ls_tolerance * |p| / scale).  Stops on scale * (cost decrease) < tolerance,
 * scale * |grad| < tolerance, a zero step, `iterations`, or (Newton) a step that left every row's
 * state unchanged -- the quadratic model was then exact and the point is the minimiser.
 * Restatement choices: the line search's stopping point, the exact-step stop, and the
 * cost decrease summed from per-row differences.  At convergence all of these reach the unique
 * minimiser of F, which is what mj_solNewton returns to within its tolerance. */
enum { ST_SAT = 0, ST_QUAD = 1, ST_LINNEG = 2, ST_LINPOS = 3 };

static int row_state(const orc_ws* w, int r, double jar) {
  if (FRIC_LIKE(w->efc_type[r])) {
    double rf = w->efc_R[r] * w->efc_frictionloss[r];
    return jar <= -rf ? ST_LINNEG : (jar >= rf ? ST_LINPOS : ST_QUAD);
  }
  return jar < 0 ? ST_QUAD : ST_SAT;
}
static double row_cost(const orc_ws* w, int r, double jar, int st) {
  double fl = w->efc_frictionloss[r];
  switch (st) {
    case ST_QUAD: return 0.5 * w->efc_D[r] * jar * jar;
    case ST_LINNEG: return -fl * jar - 0.5 * w->efc_R[r] * fl * fl;
    case ST_LINPOS: return fl * jar - 0.5 * w->efc_R[r] * fl * fl;
  }
  return 0;
}
/* cost change of a row moved from jar j0 (state s0) by dj into state s1; factored when the state is
 * kept (the GPU's fp32 form, identical in exact arithmetic) */
static double row_dcost(const orc_ws* w, int r, int s0, int s1, double j0, double dj) {
  if (s0 != s1) return row_cost(w, r, j0 + dj, s1) - row_cost(w, r, j0, s0);
  double fl = w->efc_frictionloss[r];
  return s0 == ST_QUAD ? 0.5 * w->efc_D[r] * dj * (2 * j0 + dj)
                       : (s0 == ST_LINNEG ? -fl * dj : (s0 == ST_LINPOS ? fl * dj : 0));
}
/* d cost / d jar */
static double row_slope(const orc_ws* w, int r, double jar, int st) {
  double fl = w->efc_frictionloss[r];
  return st == ST_QUAD ? w->efc_D[r] * jar : (st == ST_LINNEG ? -fl : (st == ST_LINPOS ? fl : 0));
}

static void mat_vec_n(double* y, const double* A, const double* x, int n) {
  for (int i = 0; i < n; ++i) {
    double v = 0;
    for (int k = 0; k < n; ++k) v += A[i * n + k] * x[k];
    y[i] = v;
  }
}

/* constraint update at the rows' current jar: states, forces, qfrc_constraint; returns row cost */
static double primal_update(const mrs_model_view* m, orc_ws* w) {
  int nv = m->nv, nefc = w->nefc;
  double cost = 0;
  for (int r = 0; r < nefc; ++r) {
    if (ELL_BLOCK(w, r)) {
      double c;
      const int st = ell_block(w, r, w->efc_jar + r, w->efc_force + r, &c, NULL);
      w->efc_state[r] = w->efc_state[r + 1] = w->efc_state[r + 2] = st;
      cost += c;
      r += 2;
      continue;
    }
    int st = row_state(w, r, w->efc_jar[r]);
    w->efc_state[r] = st;
    cost += row_cost(w, r, w->efc_jar[r], st);
    w->efc_force[r] = -row_slope(w, r, w->efc_jar[r], st);
  }
  for (int j = 0; j < nv; ++j) {
    double v = 0;
    for (int r = 0; r < nefc; ++r) v += w->efc_J[(size_t)r * nv + j] * w->efc_force[r];
    w->qfrc_constraint[j] = v;
  }
  return cost;
}

/* total cost at qacc x (warm-start selection) */
static double primal_cost_at(const mrs_model_view* m, orc_ws* w, const double* x, double* Mx) {
  int nv = m->nv;
  mat_vec_n(Mx, w->M, x, nv);
  double gauss = 0;
  for (int j = 0; j < nv; ++j) gauss += 0.5 * (Mx[j] - w->qfrc_smooth[j]) * (x[j] - w->qacc_smooth[j]);
  double c = 0;
  for (int r = 0; r < w->nefc; ++r) {
    const int nb = ELL_BLOCK(w, r) ? 3 : 1;
    double jar[3];
    for (int k = 0; k < nb; ++k) {
      jar[k] = -w->efc_aref[r + k];
      for (int j = 0; j < nv; ++j) jar[k] += w->efc_J[(size_t)(r + k) * nv + j] * x[j];
    }
    if (nb == 3) {
      double cb;
      ell_block(w, r, jar, NULL, &cb, NULL);
      c += cb;
      r += 2;
      continue;
    }
    c += row_cost(w, r, jar[0], row_state(w, r, jar[0]));
  }
  return gauss + c;
}

/* 1-D derivatives of F(qacc + a p) at step a; *changed: some row's state differs from step `a0` */
static void ls_eval(const orc_ws* w, double g1, double g2, double a, double a0, double* d1, double* d2,
                    int* changed) {
  double s1 = g1 + a * g2, s2 = g2;
  int ch = 0;
  for (int r = 0; r < w->nefc; ++r) {
    if (ELL_BLOCK(w, r)) {
      /* elliptic block: 1-D derivatives of its zone's cost along the line; the middle zone is not
       * quadratic in a, so a step that ends in it is never taken as exact (ch) */
      double jar[3], jv3[3];
      for (int k = 0; k < 3; ++k) { jar[k] = w->efc_jar[r + k] + a * w->efc_jv[r + k]; jv3[k] = w->efc_jv[r + k]; }
      double j0[3];
      for (int k = 0; k < 3; ++k) j0[k] = w->efc_jar[r + k] + a0 * w->efc_jv[r + k];
      const int st = ell_block(w, r, jar, NULL, NULL, NULL), st0 = ell_block(w, r, j0, NULL, NULL, NULL);
      ch |= st != st0 || st == ST_CONE;
      if (st == ST_QUAD) {
        for (int k = 0; k < 3; ++k) {
          s1 += jv3[k] * w->efc_D[r + k] * jar[k];
          s2 += w->efc_D[r + k] * jv3[k] * jv3[k];
        }
      } else if (st == ST_CONE) {
        const double mu = w->efc_mu[r], ft = w->efc_fr[r];
        const double N = mu * jar[0], dN = mu * jv3[0];
        const double U1 = ft * jar[1], U2 = ft * jar[2], dU1 = ft * jv3[1], dU2 = ft * jv3[2];
        const double T = sqrt(U1 * U1 + U2 * U2), dT = (U1 * dU1 + U2 * dU2) / T;
        const double Dm = w->efc_D[r] / (mu * mu * (1 + mu * mu)), NT = N - mu * T;
        const double g = dN - mu * dT;
        s1 += Dm * NT * g;
        s2 += Dm * (g * g - NT * mu * ((dU1 * dU1 + dU2 * dU2) - dT * dT) / T);
      }
      r += 2;
      continue;
    }
    double jv = w->efc_jv[r];
    if (jv == 0) continue;
    double jar = w->efc_jar[r] + a * jv;
    int st = row_state(w, r, jar);
    ch |= st != row_state(w, r, w->efc_jar[r] + a0 * jv);
    s1 += jv * row_slope(w, r, jar, st);
    if (st == ST_QUAD) s2 += w->efc_D[r] * jv * jv;
  }
  *d1 = s1; *d2 = s2; *changed = ch;
}

static double primal_linesearch(const mrs_model_view* m, const orc_ws* w, const double* p, const double* Mv,
                                const double* Ma, double scale) {
  int nv = m->nv;
  double snorm = 0, g1 = 0, g2 = 0;
  for (int j = 0; j < nv; ++j) {
    snorm += p[j] * p[j];
    g1 += p[j] * (Ma[j] - w->qfrc_smooth[j]);
    g2 += p[j] * Mv[j];
  }
  snorm = sqrt(snorm);
  if (snorm < MINVAL || g2 <= 0) return 0;
  double gtol = m->tolerance * m->ls_tolerance * snorm / scale;
  double a = 0, d1, d2;
  int ch;
  ls_eval(w, g1, g2, 0, 0, &d1, &d2, &ch);
  if (d1 >= 0) return 0; /* not a descent direction */
  double lo = 0, hi = -1; /* bracket: F'(lo) < 0 < F'(hi) once hi >= 0 */
  for (int it = 0; it < m->ls_iterations; ++it) {
    double an = a - d1 / d2;
    int newton = 1;
    if (hi >= 0 && (an <= lo || an >= hi)) { an = 0.5 * (lo + hi); newton = 0; }
    double n1, n2;
    ls_eval(w, g1, g2, an, a, &n1, &n2, &ch);
    a = an; d1 = n1; d2 = n2;
    if (fabs(d1) < gtol || (newton && !ch)) break;
    if (d1 < 0) lo = a; else hi = a;
  }
  return a;
}

static void solve_primal(const mrs_model_view* m, orc_data* d, int newton) {
  orc_ws* w = (orc_ws*)d->ws;
  int nv = m->nv, nefc = w->nefc;
  double scale = 1 / (m->stat_meaninertia * (nv > 1 ? nv : 1));
  size_t vb = (nv ? nv : 1) * sizeof(double);
  double *Ma = malloc(vb), *grad = malloc(vb), *Mgrad = malloc(vb), *p = malloc(vb), *Mv = malloc(vb),
         *gold = malloc(vb), *Mgold = malloc(vb), *x2 = malloc(vb);
  double *H = malloc((size_t)nv * nv * sizeof(double) + 8), *HL = malloc((size_t)nv * nv * sizeof(double) + 8);
  double* qacc = d->qacc;
  memcpy(qacc, w->qacc_smooth, vb);
  if (!(m->disableflags & MRS_DSBL_WARMSTART)) {
    /* mj_fwdConstraint: start from qacc_warmstart when its cost is not above qacc_smooth's */
    double c_ws = primal_cost_at(m, w, d->qacc_warmstart, x2);
    double c_sm = primal_cost_at(m, w, w->qacc_smooth, x2);
    if (c_ws <= c_sm) memcpy(qacc, d->qacc_warmstart, vb);
  }
  mat_vec_n(Ma, w->M, qacc, nv);
  for (int r = 0; r < nefc; ++r) {
    double jar = -w->efc_aref[r];
    for (int j = 0; j < nv; ++j) jar += w->efc_J[(size_t)r * nv + j] * qacc[j];
    w->efc_jar[r] = jar;
  }
  primal_update(m, w);
  int iter = 0, refined = 0;
  for (;;) {
    /* gradient and preconditioned gradient */
    for (int j = 0; j < nv; ++j) grad[j] = Ma[j] - w->qfrc_smooth[j] - w->qfrc_constraint[j];
    if (newton) {
      memcpy(H, w->M, (size_t)nv * nv * sizeof(double));
      for (int r = 0; r < nefc; ++r) {
        if (ELL_BLOCK(w, r)) {
          /* elliptic block: J_b' H_b J_b with the zone's 3x3 jar-space Hessian */
          double Hb[9];
          ell_block(w, r, w->efc_jar + r, NULL, NULL, Hb);
          const double* Jb = w->efc_J + (size_t)r * nv;
          for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c) {
              const double h = Hb[3 * a + c];
              if (h == 0) continue;
              for (int i = 0; i < nv; ++i)
                for (int k = 0; k < nv; ++k) H[i * nv + k] += h * Jb[(size_t)a * nv + i] * Jb[(size_t)c * nv + k];
            }
          r += 2;
          continue;
        }
        if (w->efc_state[r] != ST_QUAD) continue;
        const double* Jr = w->efc_J + (size_t)r * nv;
        for (int i = 0; i < nv; ++i)
          for (int k = 0; k < nv; ++k) H[i * nv + k] += w->efc_D[r] * Jr[i] * Jr[k];
      }
      cholesky(H, HL, nv);
      chol_solve(HL, Mgrad, grad, nv);
    } else {
      chol_solve(w->L, Mgrad, grad, nv);
    }
    if (iter == 0) {
      for (int j = 0; j < nv; ++j) p[j] = -Mgrad[j];
    } else if (newton) {
      for (int j = 0; j < nv; ++j) p[j] = -Mgrad[j];
    } else {
      double num = 0, den = 0;
      for (int j = 0; j < nv; ++j) { num += grad[j] * (Mgrad[j] - Mgold[j]); den += gold[j] * Mgold[j]; }
      double beta = num / (den > MINVAL ? den : MINVAL);
      if (beta < 0) beta = 0;
      for (int j = 0; j < nv; ++j) p[j] = -Mgrad[j] + beta * p[j];
    }
    if (iter >= m->iterations) break;
    /* line search along p */
    mat_vec_n(Mv, w->M, p, nv);
    for (int r = 0; r < nefc; ++r) {
      double v = 0;
      for (int j = 0; j < nv; ++j) v += w->efc_J[(size_t)r * nv + j] * p[j];
      w->efc_jv[r] = v;
    }
    double alpha = primal_linesearch(m, w, p, Mv, Ma, scale);
    if (alpha == 0) break;
    /* cost decrease of the step, summed from per-row differences (exact in the 1-D model) */
    double g1 = 0, g2 = 0;
    for (int j = 0; j < nv; ++j) { g1 += p[j] * (Ma[j] - w->qfrc_smooth[j]); g2 += p[j] * Mv[j]; }
    double dcost = alpha * g1 + 0.5 * alpha * alpha * g2;
    int changed = 0;
    for (int r = 0; r < nefc; ++r) {
      if (ELL_BLOCK(w, r)) {
        double j1[3], c0, c1;
        for (int k = 0; k < 3; ++k) j1[k] = w->efc_jar[r + k] + alpha * w->efc_jv[r + k];
        ell_block(w, r, w->efc_jar + r, NULL, &c0, NULL);
        const int s1 = ell_block(w, r, j1, NULL, &c1, NULL);
        dcost += c1 - c0;
        changed |= s1 != w->efc_state[r] || s1 == ST_CONE;
        for (int k = 0; k < 3; ++k) w->efc_jar[r + k] = j1[k];
        r += 2;
        continue;
      }
      double j0 = w->efc_jar[r], j1 = j0 + alpha * w->efc_jv[r];
      int s0 = w->efc_state[r], s1 = row_state(w, r, j1);
      dcost += row_dcost(w, r, s0, s1, j0, alpha * w->efc_jv[r]);
      changed |= s0 != s1;
      w->efc_jar[r] = j1;
    }
    for (int j = 0; j < nv; ++j) { qacc[j] += alpha * p[j]; Ma[j] += alpha * Mv[j]; }
    memcpy(gold, grad, vb);
    memcpy(Mgold, Mgrad, vb);
    primal_update(m, w);
    ++iter;
    double gnorm = 0;
    for (int j = 0; j < nv; ++j) {
      double g = Ma[j] - w->qfrc_smooth[j] - w->qfrc_constraint[j];
      gnorm += g * g;
    }
    if (scale * -dcost < m->tolerance || scale * sqrt(gnorm) < m->tolerance) break;
    /* mj_solNewton keeps iterating until the tests above (or the iteration count) stop it.  Opt-in
     * variant (MRS_RESTATE_NEWTON_REFINE, not upstream): */
    if (newton && !changed && (m->restate & MRS_RESTATE_NEWTON_REFINE)) {
      /* the active set held, so the step solved the quadratic model exactly up to the rounding of the
       * Hessian factor: one more step from freshly formed residuals (iterative refinement), then stop.
       * In fp64 it changes nothing measurable; in the fp32 kernel it removes the factor's rounding
       * (cond(H) eps |grad|), which otherwise shows as a residual force in the force sensors.  Skipped
       * when the residual is already within 64 eps of the gradient's own terms. */
      int above = 0; /* residual above the rounding level of the gradient's terms (DBL_EPSILON here) */
      for (int j = 0; j < nv; ++j) {
        double g = Ma[j] - w->qfrc_smooth[j] - w->qfrc_constraint[j];
        above |= fabs(g) > 64 * DBL_EPSILON * (fabs(Ma[j] - w->qfrc_smooth[j]) + fabs(w->qfrc_constraint[j]));
      }
      if (refined || !above) break;
      refined = 1;
      mat_vec_n(Ma, w->M, qacc, nv);
      for (int r = 0; r < nefc; ++r) {
        double jar = -w->efc_aref[r];
        for (int j = 0; j < nv; ++j) jar += w->efc_J[(size_t)r * nv + j] * qacc[j];
        w->efc_jar[r] = jar;
      }
      primal_update(m, w);
    }
  }
  d->solver_niter = iter;
  free(Ma); free(grad); free(Mgrad); free(p); free(Mv); free(gold); free(Mgold); free(x2); free(H); free(HL);
}

/* mj_solPGS [upstream engine_solver.c] on the dual problem
 *   min 0.5 f'AR f + f'b,  AR = J M^-1 J' + diag(R),  b = J qacc_smooth - aref,
 * friction rows boxed to [-frictionloss, frictionloss], limit/contact rows f >= 0; warm start from
 * qacc_warmstart (forces of mj_constraintUpdate), kept only if its dual cost is negative; stop when
 * the scaled cost improvement of a sweep falls below tolerance. */
static void fwd_constraint(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  int nv = m->nv, nefc = w->nefc;
  if (nefc == 0) {
    memcpy(d->qacc, w->qacc_smooth, nv * sizeof(double));
    memset(w->qfrc_constraint, 0, nv * sizeof(double));
    return;
  }
  if (m->solver != MRS_SOL_PGS) {
    solve_primal(m, d, m->solver == MRS_SOL_NEWTON);
    return;
  }
  /* M^-1 J' */
  for (int r = 0; r < nefc; ++r) chol_solve(w->L, w->efc_MinvJT + (size_t)r * nv, w->efc_J + (size_t)r * nv, nv);
  free(w->AR);
  w->AR = dalloc((size_t)nefc * nefc);
  for (int r = 0; r < nefc; ++r)
    for (int s = 0; s < nefc; ++s) {
      double v = 0;
      for (int j = 0; j < nv; ++j) v += w->efc_J[(size_t)r * nv + j] * w->efc_MinvJT[(size_t)s * nv + j];
      w->AR[(size_t)r * nefc + s] = v + (r == s ? w->efc_R[r] : 0);
    }
  for (int r = 0; r < nefc; ++r) {
    double v = 0;
    for (int j = 0; j < nv; ++j) v += w->efc_J[(size_t)r * nv + j] * w->qacc_smooth[j];
    w->efc_b[r] = v - w->efc_aref[r];
  }
  {
    /* diagnostics (scripts only): ORC_ROUND_AR=1 rounds the Delassus rows and b to fp32 (the device's
     * precision of the solver's inputs) while the iterate stays fp64 */
    static int rnd_ar = -1;
    if (rnd_ar < 0) rnd_ar = getenv("ORC_ROUND_AR") != NULL;
    if (rnd_ar) {
      for (size_t i = 0; i < (size_t)nefc * nefc; ++i) w->AR[i] = (float)w->AR[i];
      for (int r = 0; r < nefc; ++r) w->efc_b[r] = (float)w->efc_b[r];
    }
  }
  double* f = w->efc_force;
  memset(f, 0, nefc * sizeof(double));
  if (!(m->disableflags & MRS_DSBL_WARMSTART)) {
    for (int r = 0; r < nefc; ++r) {
      double jar = -w->efc_aref[r];
      for (int j = 0; j < nv; ++j) jar += w->efc_J[(size_t)r * nv + j] * d->qacc_warmstart[j];
      w->efc_jar[r] = jar;
    }
    for (int r = 0; r < nefc; ++r) {
      if (ELL_BLOCK(w, r)) {  /* elliptic block: the zone forces of mj_constraintUpdate */
        ell_block(w, r, w->efc_jar + r, f + r, NULL, NULL);
        r += 2;
        continue;
      }
      f[r] = row_force(w, r, w->efc_jar[r]);
    }
    double cost = 0;
    for (int r = 0; r < nefc; ++r) {
      double arf = 0;
      for (int s = 0; s < nefc; ++s) arf += w->AR[(size_t)r * nefc + s] * f[s];
      cost += f[r] * (0.5 * arf + w->efc_b[r]);
    }
    if (cost > 0) memset(f, 0, nefc * sizeof(double));
  }
  double scale = 1 / (m->stat_meaninertia * (nv > 1 ? nv : 1));
  d->solver_niter = 0;
  for (int it = 0; it < m->iterations; ++it) {
    double improvement = 0;
    for (int r = 0; r < nefc; ++r) {
      if (ELL_BLOCK(w, r)) {
        /* elliptic block: mj_solPGS's split update (ell_pgs_split: a normal or ray step, then the
         * friction by mju_QCQP2 with the normal fixed); opt-in MRS_RESTATE_PGS_ELLIPTIC_BLOCK instead
         * minimises the block's local cost 1/2 y'Ay + y'(res - A f_old) over the cone |y_t| <= mu y_n
         * exactly (ell_block_min) -- block Gauss-Seidel on the dual, which reaches the optimum Newton /
         * CG reach where the split update can stall on a sliding contact (the cone multiplier couples
         * normal and friction). */
        double res[3], A[9], old[3], nw[3], cb[3];
        for (int k = 0; k < 3; ++k) {
          const double* ar = w->AR + (size_t)(r + k) * nefc;
          res[k] = w->efc_b[r + k];
          for (int s = 0; s < nefc; ++s) res[k] += ar[s] * f[s];
          for (int c = 0; c < 3; ++c) A[3 * k + c] = ar[r + c];
          old[k] = f[r + k];
        }
        for (int k = 0; k < 3; ++k) cb[k] = res[k] - (A[3 * k] * old[0] + A[3 * k + 1] * old[1] + A[3 * k + 2] * old[2]);
        if (m->restate & MRS_RESTATE_PGS_ELLIPTIC_BLOCK) ell_block_min(A, cb, w->efc_fr[r], nw);
        else ell_pgs_split(A, res, old, w->efc_fr[r], nw);
        {
          /* diagnostics (scripts only): ORC_ROUND_PGS=1 rounds the block's new forces to fp32, the
           * device's storage precision, to measure how far that alone moves the iterates */
          static int rnd = -1;
          if (rnd < 0) rnd = getenv("ORC_ROUND_PGS") != NULL;
          if (rnd) for (int k = 0; k < 3; ++k) nw[k] = (float)nw[k];
        }
        double delta[3], quad = 0;
        for (int k = 0; k < 3; ++k) delta[k] = nw[k] - old[k];
        for (int k = 0; k < 3; ++k)
          for (int c = 0; c < 3; ++c) quad += delta[k] * A[3 * k + c] * delta[c];
        improvement -= delta[0] * res[0] + delta[1] * res[1] + delta[2] * res[2] + 0.5 * quad;
        for (int k = 0; k < 3; ++k) f[r + k] = nw[k];
        r += 2;
        continue;
      }
      const double* ar = w->AR + (size_t)r * nefc;
      double res = w->efc_b[r];
      for (int s = 0; s < nefc; ++s) res += ar[s] * f[s];
      double old = f[r];
      double nf = old - res / ar[r];
      if (FRIC_LIKE(w->efc_type[r])) {
        double fl = w->efc_frictionloss[r];
        nf = nf < -fl ? -fl : nf > fl ? fl : nf;
      } else if (nf < 0) {
        nf = 0;
      }
      double delta = nf - old;
      f[r] = nf;
      improvement -= delta * res + 0.5 * delta * delta * ar[r];
    }
    if (improvement * scale < m->tolerance) { d->solver_niter = it + 1; break; }
    d->solver_niter = it + 1;
  }
  for (int j = 0; j < nv; ++j) {
    double v = 0;
    for (int r = 0; r < nefc; ++r) v += w->efc_J[(size_t)r * nv + j] * f[r];
    w->qfrc_constraint[j] = v;
  }
  chol_solve(w->L, w->tmp, w->qfrc_constraint, nv);
  for (int j = 0; j < nv; ++j) d->qacc[j] = w->qacc_smooth[j] + w->tmp[j];
}

/* ------------------------------------------------------------------------ ray casting
 * mj_ray / mju_rayGeom [upstream engine_ray.c]: ray in the geom's local frame against the
 * analytic primitive; nearest non-negative hit; planes are clipped to their rendered rectangle. */
static double ray_quad(double a, double b, double c, double x[2]) {
  double det = b * b - a * c;
  if (det < MINVAL) { x[0] = x[1] = -1; return -1; }
  det = sqrt(det);
  x[0] = (-b - det) / a;
  x[1] = (-b + det) / a;
  if (x[0] >= 0) return x[0];
  if (x[1] >= 0) return x[1];
  return -1;
}
static double ray_geom_local(int type, const double* s, const double lp[3], const double lv[3]) {
  double x[2];
  switch (type) {
    case MRS_GEOM_PLANE: {
      /* parallel within 1e-6 rad or facing away: miss.  MuJoCo tests lv[2] > -mjMINVAL (1e-15);
         the relative form keeps fp32 (device) and fp64 (oracle) decisions identical for rays that
         are horizontal up to rounding (the lidar of scenes/arm7_lidar.xml). */
      if (lv[2] >= 0 || lv[2] * lv[2] <= 1e-12 * dot3(lv, lv)) return -1;
      double t = -lp[2] / lv[2];
      if (t < 0) return -1;
      double p0 = lp[0] + t * lv[0], p1 = lp[1] + t * lv[1];
      if ((s[0] <= 0 || fabs(p0) <= s[0]) && (s[1] <= 0 || fabs(p1) <= s[1])) return t;
      return -1;
    }
    case MRS_GEOM_SPHERE:
      return ray_quad(dot3(lv, lv), dot3(lv, lp), dot3(lp, lp) - s[0] * s[0], x);
    case MRS_GEOM_CAPSULE: {
      double best = -1;
      /* cylinder part */
      double a = lv[0] * lv[0] + lv[1] * lv[1];
      if (a > MINVAL) {
        double b = lv[0] * lp[0] + lv[1] * lp[1], c = lp[0] * lp[0] + lp[1] * lp[1] - s[0] * s[0];
        ray_quad(a, b, c, x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && fabs(lp[2] + x[i] * lv[2]) <= s[1] && (best < 0 || x[i] < best)) best = x[i];
      }
      /* end caps */
      for (int e = -1; e <= 1; e += 2) {
        double q[3] = {lp[0], lp[1], lp[2] - e * s[1]};
        ray_quad(dot3(lv, lv), dot3(lv, q), dot3(q, q) - s[0] * s[0], x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && e * (lp[2] + x[i] * lv[2] - e * s[1]) >= 0 && (best < 0 || x[i] < best)) best = x[i];
      }
      return best;
    }
    case MRS_GEOM_ELLIPSOID: {
      double q[3] = {lp[0] / s[0], lp[1] / s[1], lp[2] / s[2]}, v[3] = {lv[0] / s[0], lv[1] / s[1], lv[2] / s[2]};
      return ray_quad(dot3(v, v), dot3(v, q), dot3(q, q) - 1, x);
    }
    case MRS_GEOM_CYLINDER: {
      double best = -1;
      double a = lv[0] * lv[0] + lv[1] * lv[1];
      if (a > MINVAL) {
        double b = lv[0] * lp[0] + lv[1] * lp[1], c = lp[0] * lp[0] + lp[1] * lp[1] - s[0] * s[0];
        ray_quad(a, b, c, x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && fabs(lp[2] + x[i] * lv[2]) <= s[1] && (best < 0 || x[i] < best)) best = x[i];
      }
      if (fabs(lv[2]) > MINVAL)
        for (int e = -1; e <= 1; e += 2) {
          double t = (e * s[1] - lp[2]) / lv[2];
          if (t < 0) continue;
          double p0 = lp[0] + t * lv[0], p1 = lp[1] + t * lv[1];
          if (p0 * p0 + p1 * p1 <= s[0] * s[0] && (best < 0 || t < best)) best = t;
        }
      return best;
    }
    case MRS_GEOM_BOX: {
      double best = -1;
      for (int i = 0; i < 3; ++i) {
        if (fabs(lv[i]) <= MINVAL) continue;
        int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
        for (int side = -1; side <= 1; side += 2) {
          double t = (side * s[i] - lp[i]) / lv[i];
          if (t < 0) continue;
          double p1 = lp[i1] + t * lv[i1], p2 = lp[i2] + t * lv[i2];
          if (fabs(p1) <= s[i1] && fabs(p2) <= s[i2] && (best < 0 || t < best)) best = t;
        }
      }
      return best;
    }
  }
  return -1;
}
/* ray vs a mesh's triangles, both faces (mj_rayMesh): the geom's bounding box first (slab test on the
 * half extents geom_size), then every triangle (Moller-Trumbore); *tri = the nearest triangle */
static double ray_mesh(const mrs_model_view* m, int g, const double lp[3], const double lv[3], int* tri) {
  const double* s = m->geom_size + 3 * g;
  double tmin = -1e300, tmax = 1e300;
  for (int i = 0; i < 3; ++i) {
    if (fabs(lv[i]) < MINVAL) {
      if (fabs(lp[i]) > s[i]) return -1;
      continue;
    }
    double t1 = (-s[i] - lp[i]) / lv[i], t2 = (s[i] - lp[i]) / lv[i];
    if (t1 > t2) { double t = t1; t1 = t2; t2 = t; }
    tmin = fmax(tmin, t1);
    tmax = fmin(tmax, t2);
  }
  if (tmax < tmin || tmax < 0) return -1;
  int id = m->geom_dataid[g];
  const double* V = m->mesh_vert + 3 * m->mesh_vertadr[id];
  const int* F = m->mesh_face + 3 * m->mesh_faceadr[id];
  double best = -1;
  for (int f = 0; f < m->mesh_facenum[id]; ++f) {
    const double *a = V + 3 * F[3 * f], *b = V + 3 * F[3 * f + 1], *c = V + 3 * F[3 * f + 2];
    double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
    double pv[3], tv[3], qv[3];
    cross3(pv, lv, e2);
    double det = dot3(e1, pv);
    if (fabs(det) < MINVAL) continue;
    double inv = 1 / det;
    for (int i = 0; i < 3; ++i) tv[i] = lp[i] - a[i];
    double u = dot3(tv, pv) * inv;
    if (u < 0 || u > 1) continue;
    cross3(qv, tv, e1);
    double v = dot3(lv, qv) * inv;
    if (v < 0 || u + v > 1) continue;
    double t = dot3(e2, qv) * inv;
    if (t >= 0 && (best < 0 || t < best)) { best = t; if (tri) *tri = f; }
  }
  return best;
}
static double ray_geom(const mrs_model_view* m, orc_ws* w, int g, const double pnt[3], const double vec[3]) {
  const double* gp = w->geom_xpos + 3 * g;
  const double* gm = w->geom_xmat + 9 * g;
  double dv[3] = {pnt[0] - gp[0], pnt[1] - gp[1], pnt[2] - gp[2]}, lp[3], lv[3];
  matT_vec(lp, gm, dv);
  matT_vec(lv, gm, vec);
  if (m->geom_type[g] == MRS_GEOM_MESH) return ray_mesh(m, g, lp, lv, NULL);
  return ray_geom_local(m->geom_type[g], m->geom_size + 3 * g, lp, lv);
}
/* geoms a ray may hit: not on the excluded body, not fully transparent (ray_eliminate) */
static double ray_scene(const mrs_model_view* m, orc_ws* w, const double pnt[3], const double vec[3],
                        int bodyexclude, int groupmask, double tmin, int* geomid) {
  double dist = -1;
  int id = -1;
  for (int g = 0; g < m->ngeom; ++g) {
    if (m->geom_bodyid[g] == bodyexclude) continue;
    if (m->geom_rgba[4 * g + 3] == 0) continue;
    if (groupmask && !(m->geom_group[g] >= 0 && m->geom_group[g] < 6 && ((groupmask >> m->geom_group[g]) & 1))) continue;
    double t = ray_geom(m, w, g, pnt, vec);
    if (t >= tmin && (dist < 0 || t < dist)) { dist = t; id = g; }
  }
  if (geomid) *geomid = id;
  return dist;
}
double orc_ray(const mrs_model_view* m, orc_data* d, const double pnt[3], const double vec[3],
               int bodyexclude, int* geomid) {
  return ray_scene(m, (orc_ws*)d->ws, pnt, vec, bodyexclude, 0, 0, geomid);
}

/* ------------------------------------------------------------------------ sensors
 * mj_sensorPos/Vel [upstream engine_sensor.c] for the implemented types */
/* mju_transformSpatial [upstream engine_util_spatial.c]: move a com-based motion (flg_force 0) or
 * force (flg_force 1) vector [rot(3), lin(3)] from oldpos to newpos, then express it in the frame
 * rot (if given) */
static void transform_spatial(double res[6], const double vec[6], int flg_force, const double newpos[3],
                              const double oldpos[3], const double* rot) {
  double dif[3] = {newpos[0] - oldpos[0], newpos[1] - oldpos[1], newpos[2] - oldpos[2]}, cr[3], tran[6];
  memcpy(tran, vec, sizeof tran);
  if (flg_force) {
    cross3(cr, dif, vec + 3);
    for (int i = 0; i < 3; ++i) tran[i] = vec[i] - cr[i];
  } else {
    cross3(cr, dif, vec);
    for (int i = 0; i < 3; ++i) tran[3 + i] = vec[3 + i] - cr[i];
  }
  if (rot) {
    matT_vec(res, rot, tran);
    matT_vec(res + 3, rot, tran + 3);
  } else {
    memcpy(res, tran, sizeof tran);
  }
}

/* mj_rnePostConstraint [upstream engine_core_smooth.c]: cacc including qacc (world: -gravity);
 * cfrc_ext from the contact forces (mj_contactForce: pyramidal forces decoded to the contact frame,
 * rotated to world, moved to the subtree com; body2 +, body1 -); cfrc_int = cinert cacc +
 * cvel x* (cinert cvel) - cfrc_ext, summed from the leaves to the roots */
static void rne_post_constraint(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  int nb = m->nbody;
  memset(w->cacc_full, 0, 6 * sizeof(double));
  if (!(m->disableflags & MRS_DSBL_GRAVITY))
    for (int i = 0; i < 3; ++i) w->cacc_full[3 + i] = -m->gravity[i];
  memset(w->cfrc_ext, 0, 6 * (size_t)nb * sizeof(double));
  for (int c = 0; c < w->ncon; ++c) {
    const orc_contact* con = &w->con[c];
    const double* f = w->efc_force + w->efc_con_first[c];
    double lfrc[3] = {0, 0, 0};
    if (con->dim == 1) {
      lfrc[0] = f[0];
    } else if (m->cone == MRS_CONE_ELLIPTIC) {
      for (int i = 0; i < 3; ++i) lfrc[i] = f[i];  /* (normal, tangent 1, tangent 2) in the contact frame */
    } else {
      for (int i = 0; i < con->dim - 1; ++i) {
        lfrc[0] += f[2 * i] + f[2 * i + 1];
        lfrc[i + 1] = (f[2 * i] - f[2 * i + 1]) * con->friction[0];  /* tangent mu = sliding */
      }
    }
    double cfrc[6] = {0, 0, 0, 0, 0, 0}, com6[6];
    matT_vec(cfrc + 3, con->frame, lfrc); /* world force; no torsional/rolling part at condim <= 3 */
    for (int side = 0; side < 2; ++side) {
      int k = m->geom_bodyid[con->geom[side]];
      if (!k) continue;
      transform_spatial(com6, cfrc, 1, w->subtree_com + 3 * m->body_rootid[k], con->pos, NULL);
      for (int i = 0; i < 6; ++i) w->cfrc_ext[6 * k + i] += side ? com6[i] : -com6[i];
    }
  }
  memset(w->cfrc_int, 0, 6 * sizeof(double));
  for (int b = 1; b < nb; ++b) {
    double* ca = w->cacc_full + 6 * b;
    memcpy(ca, w->cacc_full + 6 * m->body_parentid[b], 6 * sizeof(double));
    int da = m->body_dofadr[b];
    for (int k = 0; k < m->body_dofnum[b]; ++k)
      for (int i = 0; i < 6; ++i)
        ca[i] += w->cdof_dot[6 * (da + k) + i] * d->qvel[da + k] + w->cdof[6 * (da + k) + i] * d->qacc[da + k];
    double f1[6], t[6], f2[6];
    mul_inert_vec(f1, w->cinert + 10 * b, ca);
    mul_inert_vec(t, w->cinert + 10 * b, w->cvel + 6 * b);
    cross_force(f2, w->cvel + 6 * b, t);
    for (int i = 0; i < 6; ++i) w->cfrc_int[6 * b + i] = f1[i] + f2[i] - w->cfrc_ext[6 * b + i];
  }
  for (int b = nb - 1; b > 0; --b)
    for (int i = 0; i < 6; ++i) w->cfrc_int[6 * m->body_parentid[b] + i] += w->cfrc_int[6 * b + i];
}

/* mj_sensorAcc for a site [upstream engine_sensor.c]: accelerometer = linear acceleration at the site
 * in the site frame (mj_objectAcceleration, local: com-based cacc/cvel moved to the site, plus
 * w x v); force / torque = cfrc_int of the site's body moved to the site, in the site frame */
static void acc_sensor(const mrs_model_view* m, orc_data* d, int type, int site, double out[3]) {
  orc_ws* w = (orc_ws*)d->ws;
  int b = m->site_bodyid[site];
  double pos[3], mat[9], v6[6], a6[6];
  site_pose(m, w, site, pos, mat);
  const double* com = w->subtree_com + 3 * m->body_rootid[b];
  if (type == MRS_SENS_ACCELEROMETER) {
    transform_spatial(v6, w->cvel + 6 * b, 0, pos, com, mat);
    transform_spatial(a6, w->cacc_full + 6 * b, 0, pos, com, mat);
    double cr[3];
    cross3(cr, v6, v6 + 3);
    for (int i = 0; i < 3; ++i) out[i] = a6[3 + i] + cr[i];
  } else {
    transform_spatial(a6, w->cfrc_int + 6 * b, 1, pos, com, mat);
    memcpy(out, type == MRS_SENS_FORCE ? a6 + 3 : a6, 3 * sizeof(double));
  }
}

static void sensors(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  if (m->disableflags & MRS_DSBL_SENSOR) return;
  for (int s = 0; s < m->nsensor; ++s) {
    int t = m->sensor_type[s];
    if (t == MRS_SENS_ACCELEROMETER || t == MRS_SENS_FORCE || t == MRS_SENS_TORQUE) {
      rne_post_constraint(m, d);
      break;
    }
  }
  for (int s = 0; s < m->nsensor; ++s) {
    double* out = d->sensordata + m->sensor_adr[s];
    int id = m->sensor_objid[s];
    switch (m->sensor_type[s]) {
      case MRS_SENS_RANGEFINDER: {
        double pos[3], mat[9];
        site_pose(m, w, id, pos, mat);
        double vec[3] = {mat[2], mat[5], mat[8]};
        out[0] = ray_scene(m, w, pos, vec, m->site_bodyid[id], 0, 0, NULL);
        break;
      }
      case MRS_SENS_JOINTPOS: out[0] = d->qpos[m->jnt_qposadr[id]]; break;
      case MRS_SENS_JOINTVEL: out[0] = d->qvel[m->jnt_dofadr[id]]; break;
      case MRS_SENS_ACTUATORFRC: out[0] = w->actuator_force[id]; break;
      case MRS_SENS_FRAMEPOS:
      case MRS_SENS_FRAMEQUAT: {
        double pos[3], q[4];
        int ot = m->sensor_objtype[s];
        if (ot == MRS_OBJ_SITE) {
          int b = m->site_bodyid[id];
          double r[3];
          rot_quat(r, m->site_pos + 3 * id, w->xquat + 4 * b);
          for (int i = 0; i < 3; ++i) pos[i] = w->xpos[3 * b + i] + r[i];
          quat_mul(q, w->xquat + 4 * b, m->site_quat + 4 * id);
        } else if (ot == MRS_OBJ_BODY) {
          memcpy(pos, w->xpos + 3 * id, sizeof pos);
          memcpy(q, w->xquat + 4 * id, sizeof q);
        } else {
          int b = m->geom_bodyid[id];
          memcpy(pos, w->geom_xpos + 3 * id, sizeof pos);
          quat_mul(q, w->xquat + 4 * b, m->geom_quat + 4 * id);
        }
        if (m->sensor_type[s] == MRS_SENS_FRAMEPOS) memcpy(out, pos, sizeof pos);
        else { quat_normalize(q); memcpy(out, q, sizeof q); }
        break;
      }
      case MRS_SENS_GYRO: {
        double pos[3], mat[9];
        site_pose(m, w, id, pos, mat);
        matT_vec(out, mat, w->cvel + 6 * m->site_bodyid[id]);
        break;
      }
      case MRS_SENS_ACCELEROMETER:
      case MRS_SENS_FORCE:
      case MRS_SENS_TORQUE: acc_sensor(m, d, m->sensor_type[s], id, out); break;
      default: memset(out, 0, m->sensor_dim[s] * sizeof(double));
    }
    if (m->sensor_cutoff[s] > 0 && m->sensor_type[s] != MRS_SENS_RANGEFINDER &&
        m->sensor_type[s] != MRS_SENS_FRAMEQUAT)
      for (int i = 0; i < m->sensor_dim[s]; ++i) {
        double c = m->sensor_cutoff[s];
        out[i] = out[i] < -c ? -c : out[i] > c ? c : out[i];
      }
  }
}

/* ------------------------------------------------------------------------ forward / step */
static void fwd_position(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  kinematics(m, d);
  com_pos(m, d);
  make_M(m, d);
  cholesky(w->M, w->L, m->nv);
  collision(m, d);
  make_constraint(m, d);
}

/* mj_forwardSkip(m, d, mjSTAGE_NONE, skip_sensor) */
static void forward_skip(const mrs_model_view* m, orc_data* d, int skip_sensor) {
  orc_ws* w = (orc_ws*)d->ws;
  int nv = m->nv;
  fwd_position(m, d);
  com_vel(m, d);
  passive(m, d);
  rne(m, d);
  actuation(m, d);
  for (int j = 0; j < nv; ++j)
    w->qfrc_smooth[j] = w->qfrc_passive[j] - w->qfrc_bias[j] + d->qfrc_applied[j] + d->qfrc_actuator[j];
  chol_solve(w->L, w->qacc_smooth, w->qfrc_smooth, nv);
  /* constraint impedance/aref need efc_vel from qvel: recompute after comVel (rows built above) */
  fwd_constraint(m, d);
  if (!skip_sensor) sensors(m, d);
  d->ncon = w->ncon;
  d->nefc = w->nefc;
}

void orc_forward(const mrs_model_view* m, orc_data* d) { forward_skip(m, d, 0); }

/* mj_integratePos: qpos advanced by h * vel (free joints: position and quaternion; ball: quaternion) */
static void integrate_pos(const mrs_model_view* m, double* qpos, const double* vel, double h) {
  for (int j = 0; j < m->njnt; ++j) {
    int a = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    switch (m->jnt_type[j]) {
      case MRS_JNT_FREE:
        for (int i = 0; i < 3; ++i) qpos[a + i] += h * vel[da + i];
        a += 3; da += 3;
        /* fall through */
      case MRS_JNT_BALL: {
        double* q = qpos + a;
        double v[3] = {vel[da], vel[da + 1], vel[da + 2]};
        double ang = h * normalize3(v);
        double dq[4];
        axis_angle_quat(dq, v, ang);
        quat_normalize(q);
        quat_mul(q, q, dq);
        quat_normalize(q);
        break;
      }
      default: qpos[a] += h * vel[da];
    }
  }
}

/* mj_Euler (implicit in joint damping) and mj_implicit (implicitfast / implicit) [upstream
 * engine_forward.c]:
 *   (M + h*diag(B_eff) [+ h dB]) qacc_int = qfrc_smooth + qfrc_constraint
 * with B_eff = dof damping (Euler) or dof damping - d(actuator force)/d(qvel) (implicitfast; joint
 * transmissions make it diagonal), dB = d qfrc_bias / d qvel for the full implicit integrator
 * (orc_bias_vel), then qvel += h qacc_int, integrate qpos, time += h. */
/* qfrc_bias (mj_rne, flg_acc = 0) at velocity v with the current positions: com_vel + rne on v, the
 * velocity-dependent work arrays and qvel restored after */
static void bias_at(const mrs_model_view* m, orc_data* d, const double* v, double* out) {
  orc_ws* w = (orc_ws*)d->ws;
  const int nb = m->nbody, nv = m->nv;
  double* save = (double*)malloc(sizeof(double) * (size_t)(24 * nb + 6 * nv + 2 * nv + 1));
  double* p = save;
  memcpy(p, w->cvel, 6 * nb * sizeof(double)); p += 6 * nb;
  memcpy(p, w->cacc, 6 * nb * sizeof(double)); p += 6 * nb;
  memcpy(p, w->cfrc, 6 * nb * sizeof(double)); p += 6 * nb;
  memcpy(p, w->cdof_dot, 6 * nv * sizeof(double)); p += 6 * nv;
  memcpy(p, w->qfrc_bias, nv * sizeof(double)); p += nv;
  memcpy(p, d->qvel, nv * sizeof(double));
  memcpy(d->qvel, v, nv * sizeof(double));
  com_vel(m, d);
  rne(m, d);
  memcpy(out, w->qfrc_bias, nv * sizeof(double));
  p = save;
  memcpy(w->cvel, p, 6 * nb * sizeof(double)); p += 6 * nb;
  memcpy(w->cacc, p, 6 * nb * sizeof(double)); p += 6 * nb;
  memcpy(w->cfrc, p, 6 * nb * sizeof(double)); p += 6 * nb;
  memcpy(w->cdof_dot, p, 6 * nv * sizeof(double)); p += 6 * nv;
  memcpy(w->qfrc_bias, p, nv * sizeof(double)); p += nv;
  memcpy(d->qvel, p, nv * sizeof(double));
  free(save);
}

/* mjd_rne_vel restated: dB[i * nv + j] = d qfrc_bias_i / d qvel_j.  qfrc_bias = C(q, v) v + g(q) is
 * exactly quadratic in v for fixed positions (Coriolis, centrifugal and gyroscopic terms; gravity is
 * constant), so the central difference (B(v + e_j) - B(v - e_j)) / 2 is its derivative with no
 * truncation error, only rounding -- the same matrix upstream's analytic recursion forms
 * [restated; verify]. */
void orc_bias_vel(const mrs_model_view* m, orc_data* d, double* dB) {
  const int nv = m->nv;
  double* v = (double*)malloc(sizeof(double) * (size_t)(3 * nv + 1));
  double *bp = v + nv, *bm = bp + nv;
  for (int j = 0; j < nv; ++j) {
    memcpy(v, d->qvel, nv * sizeof(double));
    v[j] += 1;
    bias_at(m, d, v, bp);
    v[j] -= 2;
    bias_at(m, d, v, bm);
    for (int i = 0; i < nv; ++i) dB[i * nv + j] = 0.5 * (bp[i] - bm[i]);
  }
  free(v);
}

/* dense LU without pivoting (mj_factorLU restated densely: the implicit matrix is M plus small h-scaled
 * derivative terms, so it stays diagonally dominated like M) and the solve A x = b, in place */
static void lu_solve(double* A, double* x, const double* b, int n) {
  for (int k = 0; k < n; ++k)
    for (int i = k + 1; i < n; ++i) {
      const double l = A[i * n + k] / A[k * n + k];
      A[i * n + k] = l;
      for (int j = k + 1; j < n; ++j) A[i * n + j] -= l * A[k * n + j];
    }
  for (int i = 0; i < n; ++i) {
    double v = b[i];
    for (int k = 0; k < i; ++k) v -= A[i * n + k] * x[k];
    x[i] = v;
  }
  for (int i = n - 1; i >= 0; --i) {
    double v = x[i];
    for (int k = i + 1; k < n; ++k) v -= A[i * n + k] * x[k];
    x[i] = v / A[i * n + i];
  }
}

static void integrate(const mrs_model_view* m, orc_data* d) {
  orc_ws* w = (orc_ws*)d->ws;
  int nv = m->nv;
  double h = m->timestep;
  double* qacc_int = w->tmp;
  int need_solve = 0;
  double* Dg = (double*)calloc(nv ? nv : 1, sizeof(double));
  if (m->integrator == MRS_INT_EULER) {
    if (!(m->disableflags & MRS_DSBL_EULERDAMP))
      for (int j = 0; j < nv; ++j) if (m->dof_damping[j] > 0) { Dg[j] = m->dof_damping[j]; need_solve = 1; }
  } else { /* implicitfast, implicit */
    need_solve = 1;
    if (!(m->disableflags & MRS_DSBL_PASSIVE))
      for (int j = 0; j < nv; ++j) Dg[j] = m->dof_damping[j];
    if (!(m->disableflags & MRS_DSBL_ACTUATION))
      for (int a = 0; a < m->nu; ++a) {
        /* (tendon actuators on these integrators have no velocity term: the compiler requires it) */
        if (m->actuator_trntype[a] == MRS_TRN_TENDON) continue;
        if (m->actuator_forcelimited[a]) {
          double f = w->actuator_force[a];
          const double* r = m->actuator_forcerange + 2 * a;
          if (f <= r[0] || f >= r[1]) continue;
        }
        double bv = m->actuator_biastype[a] == MRS_BIAS_AFFINE ? m->actuator_biasprm[MRS_NBIAS * a + 2] : 0;
        double gv = m->actuator_gaintype[a] == MRS_GAIN_AFFINE ? m->actuator_gainprm[MRS_NGAIN * a + 2] : 0;
        double ctrl = d->ctrl[a];
        if (m->actuator_ctrllimited[a] && !(m->disableflags & MRS_DSBL_CLAMPCTRL)) {
          const double* r = m->actuator_ctrlrange + 2 * a;
          ctrl = ctrl < r[0] ? r[0] : ctrl > r[1] ? r[1] : ctrl;
        }
        double v = bv + gv * ctrl;
        double gear = m->actuator_gear[6 * a];
        Dg[m->jnt_dofadr[m->actuator_trnid[2 * a]]] -= gear * gear * v;
      }
  }
  if (need_solve && m->integrator == MRS_INT_IMPLICIT) {
    /* mj_implicit: (M - h qDeriv) qacc_int = qfrc_smooth + qfrc_constraint with the full velocity
     * derivative qDeriv = d(qfrc_passive + qfrc_actuator - qfrc_bias)/d qvel: the diagonal terms of
     * implicitfast plus the RNE (Coriolis / centrifugal / gyroscopic) derivative, non-symmetric, so LU */
    memcpy(w->Mi, w->M, (size_t)nv * nv * sizeof(double));
    orc_bias_vel(m, d, w->Li);
    for (int i = 0; i < nv; ++i)
      for (int j = 0; j < nv; ++j) w->Mi[i * nv + j] += h * w->Li[i * nv + j];
    for (int j = 0; j < nv; ++j) w->Mi[j * nv + j] += h * Dg[j];
    for (int j = 0; j < nv; ++j) w->tmp2[j] = w->qfrc_smooth[j] + w->qfrc_constraint[j];
    lu_solve(w->Mi, qacc_int, w->tmp2, nv);
  } else if (need_solve) {
    memcpy(w->Mi, w->M, (size_t)nv * nv * sizeof(double));
    for (int j = 0; j < nv; ++j) w->Mi[j * nv + j] += h * Dg[j];
    cholesky(w->Mi, w->Li, nv);
    for (int j = 0; j < nv; ++j) w->tmp2[j] = w->qfrc_smooth[j] + w->qfrc_constraint[j];
    chol_solve(w->Li, qacc_int, w->tmp2, nv);
  } else {
    memcpy(qacc_int, d->qacc, nv * sizeof(double));
  }
  free(Dg);
  /* mj_advance: warm start keeps the constraint solver's qacc */
  memcpy(d->qacc_warmstart, d->qacc, nv * sizeof(double));
  for (int j = 0; j < nv; ++j) d->qvel[j] += h * qacc_int[j];
  integrate_pos(m, d->qpos, d->qvel, h);
  d->time += h;
}

/* mj_RungeKutta(m, d, 4) [upstream engine_forward.c], restated: the classic tableau A = diag(1/2, 1/2,
 * 1), B = (1/6, 1/3, 1/3, 1/6), C = (1/2, 1/2, 1).  F_0 = (qvel, qacc) of the step's mj_forward; stage
 * i = 1..3 sets X_i = X_0 '+' h A_i F_{i-1} (positions by mj_integratePos with velocity A_i qvel_{i-1},
 * velocities qvel_0 + h A_i qacc_{i-1}) and evaluates F_i by mj_forwardSkip without sensors; then the
 * state returns to X_0 and mj_advance moves it by h sum_j B_j F_j (qvel += h dX_acc, positions
 * integrated with dX_vel), qacc_warmstart = the last stage's qacc [restated; verify against upstream].
 * Sensor data stays that of the step's first forward, the other mjData outputs are the last stage's. */
static void rk4(const mrs_model_view* m, orc_data* d) {
  static const double A[3] = {0.5, 0.5, 1.0}, B[4] = {1.0 / 6, 1.0 / 3, 1.0 / 3, 1.0 / 6};
  const int nq = m->nq, nv = m->nv;
  const double h = m->timestep, t0 = d->time;
  double* q0 = (double*)malloc((size_t)(nq ? nq : 1) * sizeof(double));
  double* buf = (double*)calloc((size_t)(4 * nv + 1), sizeof(double));
  double *v0 = buf, *sv = buf + nv, *sa = buf + 2 * nv, *dv = buf + 3 * nv;
  memcpy(q0, d->qpos, nq * sizeof(double));
  memcpy(v0, d->qvel, nv * sizeof(double));
  for (int i = 1; i < 4; ++i) {
    for (int j = 0; j < nv; ++j) {
      const double vel = d->qvel[j], acc = d->qacc[j];
      sv[j] += B[i - 1] * vel;
      sa[j] += B[i - 1] * acc;
      dv[j] = A[i - 1] * vel;
      d->qvel[j] = v0[j] + h * (A[i - 1] * acc);
    }
    memcpy(d->qpos, q0, nq * sizeof(double));
    integrate_pos(m, d->qpos, dv, h);
    d->time = t0 + A[i - 1] * h;
    forward_skip(m, d, 1);
  }
  for (int j = 0; j < nv; ++j) {
    sv[j] += B[3] * d->qvel[j];
    sa[j] += B[3] * d->qacc[j];
  }
  memcpy(d->qpos, q0, nq * sizeof(double));
  /* mj_advance */
  memcpy(d->qacc_warmstart, d->qacc, nv * sizeof(double));
  for (int j = 0; j < nv; ++j) d->qvel[j] = v0[j] + h * sa[j];
  integrate_pos(m, d->qpos, sv, h);
  d->time = t0 + h;
  free(q0);
  free(buf);
}

/* mj_checkPos / mj_checkVel / mj_checkAcc with auto-reset [upstream engine_forward.c] */
static int check(const mrs_model_view* m, orc_data* d, const double* x, int n, int which) {
  for (int i = 0; i < n; ++i)
    if (is_bad(x[i])) {
      d->warning[which]++;
      d->warning[3] = i;
      if (!(m->disableflags & MRS_DSBL_AUTORESET)) {
        int w0 = d->warning[0], w1 = d->warning[1], w2 = d->warning[2], w3 = d->warning[3];
        orc_reset(m, d, -1);
        d->warning[0] = w0; d->warning[1] = w1; d->warning[2] = w2; d->warning[3] = w3;
      }
      return 1;
    }
  return 0;
}

void orc_step(const mrs_model_view* m, orc_data* d) {
  check(m, d, d->qpos, m->nq, 0);
  check(m, d, d->qvel, m->nv, 1);
  orc_forward(m, d);
  if (check(m, d, d->qacc, m->nv, 2)) orc_forward(m, d);
  if (m->integrator == MRS_INT_RK4) rk4(m, d);
  else integrate(m, d);
}

void orc_mass_matrix(const mrs_model_view* m, orc_data* d, double* M) {
  orc_ws* w = (orc_ws*)d->ws;
  kinematics(m, d);
  com_pos(m, d);
  make_M(m, d);
  memcpy(M, w->M, (size_t)m->nv * m->nv * sizeof(double));
}

void orc_kinematics(const mrs_model_view* m, orc_data* d, double* xpos, double* xquat,
                    double* geom_xpos, double* geom_xmat) {
  orc_ws* w = (orc_ws*)d->ws;
  kinematics(m, d);
  com_pos(m, d);
  if (xpos) memcpy(xpos, w->xpos, 3 * m->nbody * sizeof(double));
  if (xquat) memcpy(xquat, w->xquat, 4 * m->nbody * sizeof(double));
  if (geom_xpos) memcpy(geom_xpos, w->geom_xpos, 3 * m->ngeom * sizeof(double));
  if (geom_xmat) memcpy(geom_xmat, w->geom_xmat, 9 * m->ngeom * sizeof(double));
}

/* debugging / tests: constraint rows of the last forward (type, force, aref, R, pos, J) */
int orc_efc(orc_data* d, int nv, int max, int* type, double* force, double* aref, double* R, double* pos,
            double* J) {
  orc_ws* w = (orc_ws*)d->ws;
  int n = w->nefc < max ? w->nefc : max;
  for (int r = 0; r < n; ++r) {
    type[r] = w->efc_type[r]; force[r] = w->efc_force[r]; aref[r] = w->efc_aref[r];
    R[r] = w->efc_R[r]; pos[r] = w->efc_pos[r];
    memcpy(J + (size_t)r * nv, w->efc_J + (size_t)r * nv, nv * sizeof(double));
  }
  return w->nefc;
}

/* qacc_smooth and qfrc_smooth of the last forward (tests) */
void orc_smooth(const mrs_model_view* m, orc_data* d, double* qacc_smooth, double* qfrc_smooth) {
  orc_ws* w = (orc_ws*)d->ws;
  memcpy(qacc_smooth, w->qacc_smooth, m->nv * sizeof(double));
  memcpy(qfrc_smooth, w->qfrc_smooth, m->nv * sizeof(double));
}

int orc_contacts(orc_data* d, int max, int* geom, double* dist, double* pos, double* frame) {
  orc_ws* w = (orc_ws*)d->ws;
  int n = w->ncon < max ? w->ncon : max;
  for (int c = 0; c < n; ++c) {
    if (geom) { geom[2 * c] = w->con[c].geom[0]; geom[2 * c + 1] = w->con[c].geom[1]; }
    if (dist) dist[c] = w->con[c].dist;
    if (pos) memcpy(pos + 3 * c, w->con[c].pos, 3 * sizeof(double));
    if (frame) memcpy(frame + 9 * c, w->con[c].frame, 9 * sizeof(double));
  }
  return w->ncon;
}

/* ------------------------------------------------------------------------ depth camera
 * Replaces mjr_render + mjr_readPixels + linearisation (src/mujoco_cameras.cpp:211-240): one ray
 * per pixel centre through the pinhole (fovy, H; fx = fy = H/2 / tan(fovy/2) as in the plugin's
 * intrinsics :119-123), eye-space depth = ray parameter along the camera -z axis, geoms of groups
 * 0-2 (mjvOption default), hits nearer than znear*extent ignored, misses -> far = zfar*extent.
 * Row 0 is the top row (the plugin's vertical flip, :229-240, already applied). */
/* colour of a hit: flat headlight shading rgba * (0.3 + 0.7 max(0, -n.d)) of the geom's surface
 * normal n at the hit and the unit pixel ray d (the device's batch.hip local_normal / shade).  Not a
 * restatement of the reference's OpenGL render (src/mujoco_cameras.cpp:211-240): parity unpinned
 * against the reference, pinned between device and this oracle. */
static void local_normal(int type, const double* s, const double p[3], double n[3]) {
  n[0] = 0; n[1] = 0; n[2] = 1;
  switch (type) {
    case MRS_GEOM_SPHERE: n[0] = p[0]; n[1] = p[1]; n[2] = p[2]; break;
    case MRS_GEOM_CAPSULE: {
      double z = p[2] < -s[1] ? -s[1] : (p[2] > s[1] ? s[1] : p[2]);
      n[0] = p[0]; n[1] = p[1]; n[2] = p[2] - z;
      break;
    }
    case MRS_GEOM_ELLIPSOID: n[0] = p[0] / (s[0] * s[0]); n[1] = p[1] / (s[1] * s[1]); n[2] = p[2] / (s[2] * s[2]); break;
    case MRS_GEOM_CYLINDER: {
      double rr = sqrt(p[0] * p[0] + p[1] * p[1]);
      if (fabs(p[2]) - s[1] > rr - s[0]) { n[0] = 0; n[1] = 0; n[2] = p[2] >= 0 ? 1 : -1; }
      else { n[0] = p[0]; n[1] = p[1]; n[2] = 0; }
      break;
    }
    case MRS_GEOM_BOX: {
      int k = 0;
      double best = fabs(p[0]) / s[0];
      for (int i = 1; i < 3; ++i)
        if (fabs(p[i]) / s[i] > best) { best = fabs(p[i]) / s[i]; k = i; }
      n[0] = n[1] = n[2] = 0;
      n[k] = p[k] >= 0 ? 1 : -1;
      break;
    }
    default: break;
  }
}

/* ---- colour [restated from MuJoCo's OpenGL renderer (mjr_render: fixed-function lighting, materials,
 * builtin textures, shadows, skybox); verify]: per pixel (not per vertex), per light l (the headlight
 * first -- a directional light along the view axis with vis.headlight's colours, no shadow -- then the
 * model's active lights, fixed in the world):
 *   c = emission base + sum_l att_l spot_l (amb_l base + sh_l (max(0, N.L) diff_l base
 *                                                               + [N.L > 0] max(0, N.H)^(128 shininess) spec_l specular))
 * N the surface normal facing the viewer, L towards the light, H = normalize(L + E) with E the view
 * axis (OpenGL's infinite viewer), att = 1 / (a0 + a1 d + a2 d^2) and spot = cos^exponent inside the
 * cutoff cone for spot lights (1 for directional ones), sh_l = 0 when the ray from the surface (offset
 * 1e-4 along N) towards the light hits a geom of groups 0-2 first (castshadow lights).  base = rgba,
 * times the 2-D texture for planes (texcoords = the plane-frame hit x, y times texrepeat, per unit
 * length when texuniform, else per plane size; nearest texel of the builtin image: 2 x 2 checker
 * rgb1 / rgb2, vertical gradient rgb1 -> rgb2 or flat rgb1, marks edge / cross in markrgb).  Material
 * defaults without one: specular 0.5, shininess 0.5, emission 0.  A miss shows the first skybox
 * texture (gradient: rgb2 + (rgb1 - rgb2) (1 + d_z) / 2 of the world view direction; flat / checker:
 * rgb1 above the horizon, rgb2 below), else black.  Channels clamped to [0, 1], rounded to 8 bits. */
static void tex_sample(const mrs_model_view* m, int t, double u, double v, double out[3]) {
  const int W = m->tex_width[t], H = m->tex_height[t];
  u -= floor(u);
  v -= floor(v);
  int iu = (int)(u * W), iv = (int)(v * H);
  iu = iu < 0 ? 0 : (iu >= W ? W - 1 : iu);
  iv = iv < 0 ? 0 : (iv >= H ? H - 1 : iv);
  const double *c1 = m->tex_rgb1 + 3 * t, *c2 = m->tex_rgb2 + 3 * t;
  switch (m->tex_builtin[t]) {
    case MRS_BUILTIN_CHECKER: {
      const double* c = ((iu < W / 2) == (iv < H / 2)) ? c1 : c2;
      for (int i = 0; i < 3; ++i) out[i] = c[i];
      break;
    }
    case MRS_BUILTIN_GRADIENT: {
      const double s = H > 1 ? (double)iv / (H - 1) : 0;
      for (int i = 0; i < 3; ++i) out[i] = c1[i] + s * (c2[i] - c1[i]);
      break;
    }
    default:
      for (int i = 0; i < 3; ++i) out[i] = c1[i];
  }
  const int mk = m->tex_mark[t];
  if ((mk == MRS_MARK_EDGE && (iu == 0 || iv == 0 || iu == W - 1 || iv == H - 1)) ||
      (mk == MRS_MARK_CROSS && (iu == W / 2 || iv == H / 2)))
    for (int i = 0; i < 3; ++i) out[i] = m->tex_markrgb[3 * t + i];
}
static void sky_color(const mrs_model_view* m, const double dir[3], double out[3]) {
  out[0] = out[1] = out[2] = 0;
  for (int t = 0; t < m->ntex; ++t) {
    if (m->tex_type[t] != MRS_TEX_SKYBOX) continue;
    const double dz = dir[2] / sqrt(dot3(dir, dir));
    const double *c1 = m->tex_rgb1 + 3 * t, *c2 = m->tex_rgb2 + 3 * t;
    if (m->tex_builtin[t] == MRS_BUILTIN_GRADIENT)
      for (int i = 0; i < 3; ++i) out[i] = c2[i] + (c1[i] - c2[i]) * 0.5 * (1 + dz);
    else
      for (int i = 0; i < 3; ++i) out[i] = dz >= 0 ? c1[i] : c2[i];
    return;
  }
}
static void lit_color(const mrs_model_view* m, orc_ws* w, int g, const double P[3], const double nw[3],
                      const double vec[3], const double q[3], const double E[3], double out[3]) {
  double N[3] = {nw[0], nw[1], nw[2]}, base[3], spec_m = 0.5, shin = 0.5, emis = 0;
  normalize3(N);
  if (dot3(N, vec) > 0) for (int i = 0; i < 3; ++i) N[i] = -N[i];
  for (int i = 0; i < 3; ++i) base[i] = m->geom_rgba[4 * g + i];
  const int mat = m->nmat ? m->geom_matid[g] : -1;
  if (mat >= 0) {
    spec_m = m->mat_specular[mat]; shin = m->mat_shininess[mat]; emis = m->mat_emission[mat];
    const int t = m->mat_texid[mat];
    if (t >= 0 && m->tex_type[t] == MRS_TEX_2D && m->geom_type[g] == MRS_GEOM_PLANE) {
      double sc[2];
      for (int k = 0; k < 2; ++k) {
        const double sz = m->geom_size[3 * g + k];
        sc[k] = m->mat_texrepeat[2 * mat + k] * (m->mat_texuniform[mat] || sz <= 0 ? 1.0 : 1.0 / (2 * sz));
      }
      double tc[3];
      tex_sample(m, t, q[0] * sc[0], q[1] * sc[1], tc);
      for (int i = 0; i < 3; ++i) base[i] *= tc[i];
    }
  }
  for (int i = 0; i < 3; ++i) out[i] = emis * base[i];
  for (int l = -1; l < m->nlight; ++l) {
    double L[3], amb[3], dif[3], spc[3], att = 1, spot = 1, dist = 1e300;
    int shadow = 0;
    if (l < 0) {
      if (!m->vis_headlight[9]) continue;
      for (int i = 0; i < 3; ++i) {
        L[i] = E[i]; amb[i] = m->vis_headlight[i]; dif[i] = m->vis_headlight[3 + i]; spc[i] = m->vis_headlight[6 + i];
      }
    } else {
      if (!m->light_active[l]) continue;
      const double* dir = m->light_dir + 3 * l;
      for (int i = 0; i < 3; ++i) {
        amb[i] = m->light_ambient[3 * l + i]; dif[i] = m->light_diffuse[3 * l + i]; spc[i] = m->light_specular[3 * l + i];
      }
      shadow = m->light_castshadow[l];
      if (m->light_directional[l]) {
        for (int i = 0; i < 3; ++i) L[i] = -dir[i];
      } else {
        for (int i = 0; i < 3; ++i) L[i] = m->light_pos[3 * l + i] - P[i];
        dist = normalize3(L);
        const double* a = m->light_attenuation + 3 * l;
        att = 1 / (a[0] + a[1] * dist + a[2] * dist * dist);
        const double ca = -dot3(L, dir);
        spot = ca < cos(m->light_cutoff[l] * M_PI / 180) ? 0 : pow(ca, m->light_exponent[l]);
      }
      normalize3(L);
    }
    const double nl = fmax(0, dot3(N, L));
    double sh = 1;
    if (shadow && nl > 0) {
      double o[3];
      for (int i = 0; i < 3; ++i) o[i] = P[i] + 1e-4 * N[i];
      const double th = ray_scene(m, w, o, L, -1, 0x7, 0, NULL);
      if (th >= 0 && th < dist) sh = 0;
    }
    double H[3] = {L[0] + E[0], L[1] + E[1], L[2] + E[2]};
    normalize3(H);
    const double sp = nl > 0 ? pow(fmax(0, dot3(N, H)), 128 * shin) : 0;
    for (int i = 0; i < 3; ++i)
      out[i] += att * spot * (amb[i] * base[i] + sh * (nl * dif[i] * base[i] + sp * spc[i] * spec_m));
  }
}

void orc_render_rgbd(const mrs_model_view* m, orc_data* d, int cam, float* depth, unsigned char* rgb) {
  orc_ws* w = (orc_ws*)d->ws;
  kinematics(m, d);
  int W = m->cam_resolution[2 * cam], H = m->cam_resolution[2 * cam + 1];
  int b = m->cam_bodyid[cam];
  double cpos[3], cq[4], cmat[9], r[3];
  rot_quat(r, m->cam_pos + 3 * cam, w->xquat + 4 * b);
  for (int i = 0; i < 3; ++i) cpos[i] = w->xpos[3 * b + i] + r[i];
  quat_mul(cq, w->xquat + 4 * b, m->cam_quat + 4 * cam);
  quat2mat(cmat, cq);
  double znear = m->vis_znear * m->stat_extent, zfar = m->vis_zfar * m->stat_extent;
  double f = 0.5 * H / tan(m->cam_fovy[cam] * M_PI / 360.0);
  for (int row = 0; row < H; ++row)
    for (int col = 0; col < W; ++col) {
      double dc[3] = {(col + 0.5 - 0.5 * W) / f, (0.5 * H - row - 0.5) / f, -1}, vec[3];
      mat_vec(vec, cmat, dc);
      int g = -1;
      double t = ray_scene(m, w, cpos, vec, -1, 0x7, znear, &g);
      int hit = !(t < 0 || t > zfar);
      if (depth) depth[(size_t)row * W + col] = (float)(hit ? t : zfar);
      if (!rgb) continue;
      unsigned char* px = rgb + ((size_t)row * W + col) * 3;
      double cl[3];
      if (!hit) {
        sky_color(m, vec, cl);
        for (int ch = 0; ch < 3; ++ch) px[ch] = (unsigned char)(fmin(fmax(cl[ch], 0), 1) * 255.0 + 0.5);
        continue;
      }
      const double* gm = w->geom_xmat + 9 * g;
      double dv[3], q[3], lv[3], nl[3], nw[3];
      for (int i = 0; i < 3; ++i) dv[i] = cpos[i] + t * vec[i] - w->geom_xpos[3 * g + i];
      matT_vec(q, gm, dv);
      if (m->geom_type[g] == MRS_GEOM_MESH) {  /* the hit triangle's normal */
        double lpc[3], dc2[3];
        int tri = 0;
        for (int i = 0; i < 3; ++i) dc2[i] = cpos[i] - w->geom_xpos[3 * g + i];
        matT_vec(lpc, gm, dc2);
        matT_vec(lv, gm, vec);
        ray_mesh(m, g, lpc, lv, &tri);
        int id = m->geom_dataid[g];
        const double* V = m->mesh_vert + 3 * m->mesh_vertadr[id];
        const int* F = m->mesh_face + 3 * (m->mesh_faceadr[id] + tri);
        double e1[3], e2[3];
        for (int i = 0; i < 3; ++i) { e1[i] = V[3 * F[1] + i] - V[3 * F[0] + i]; e2[i] = V[3 * F[2] + i] - V[3 * F[0] + i]; }
        cross3(nl, e1, e2);
        if (dot3(nl, lv) > 0) for (int i = 0; i < 3; ++i) nl[i] = -nl[i];  /* two-sided */
      } else {
        local_normal(m->geom_type[g], m->geom_size + 3 * g, q, nl);
      }
      mat_vec(nw, gm, nl);
      double P[3], E[3] = {cmat[2], cmat[5], cmat[8]};
      for (int i = 0; i < 3; ++i) P[i] = cpos[i] + t * vec[i];
      lit_color(m, w, g, P, nw, vec, q, E, cl);
      for (int ch = 0; ch < 3; ++ch) px[ch] = (unsigned char)(fmin(fmax(cl[ch], 0), 1) * 255.0 + 0.5);
    }
}

void orc_render_depth(const mrs_model_view* m, orc_data* d, int cam, float* out) {
  orc_render_rgbd(m, d, cam, out, NULL);
}

/* ------------------------------------------------------------------------ CPU baseline */
typedef struct {
  const mrs_model_view* m;
  int env0, env1, n_steps, period, n_envs, cpu;
  const double *ctrl_table, *qpos_init;
  double *qpos_out, *qvel_out;
} rollout_job;

static void* rollout_worker(void* arg) {
  rollout_job* j = (rollout_job*)arg;
  const mrs_model_view* m = j->m;
  if (j->cpu >= 0) { /* one worker per allowed CPU, pinned */
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(j->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof set, &set);
  }
  orc_data* d = orc_make_data(m);
  for (int e = j->env0; e < j->env1; ++e) {
    orc_reset(m, d, -1);
    if (j->qpos_init) memcpy(d->qpos, j->qpos_init + (size_t)e * m->nq, m->nq * sizeof(double));
    for (int t = 0; t < j->n_steps; ++t) {
      if (t % j->period == 0 && j->ctrl_table)
        memcpy(d->ctrl, j->ctrl_table + ((size_t)(t / j->period) * j->n_envs + e) * m->nu, m->nu * sizeof(double));
      orc_step(m, d);
    }
    if (j->qpos_out) memcpy(j->qpos_out + (size_t)e * m->nq, d->qpos, m->nq * sizeof(double));
    if (j->qvel_out) memcpy(j->qvel_out + (size_t)e * m->nv, d->qvel, m->nv * sizeof(double));
  }
  orc_free_data(d);
  return NULL;
}

double orc_rollout(const mrs_model_view* m, int n_envs, int n_steps, int period,
                   const double* ctrl_table, const double* qpos_init, int n_threads,
                   double* qpos_out, double* qvel_out) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > n_envs) n_threads = n_envs;
  pthread_t th[256];
  rollout_job jobs[256];
  if (n_threads > 256) n_threads = 256;
  /* the CPUs this process may run on, in order: worker i is pinned to the i-th of them when there
   * are at least as many CPUs as workers */
  int cpus[256], ncpu = 0;
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof allowed, &allowed) == 0)
    for (int c = 0; c < CPU_SETSIZE && ncpu < 256; ++c)
      if (CPU_ISSET(c, &allowed)) cpus[ncpu++] = c;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int i = 0; i < n_threads; ++i) {
    rollout_job* j = &jobs[i];
    j->cpu = ncpu >= n_threads ? cpus[i] : -1;
    j->m = m; j->n_steps = n_steps; j->period = period > 0 ? period : 1; j->n_envs = n_envs;
    j->ctrl_table = ctrl_table; j->qpos_init = qpos_init; j->qpos_out = qpos_out; j->qvel_out = qvel_out;
    j->env0 = (int)((long)n_envs * i / n_threads);
    j->env1 = (int)((long)n_envs * (i + 1) / n_threads);
    pthread_create(&th[i], NULL, rollout_worker, j);
  }
  for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}
