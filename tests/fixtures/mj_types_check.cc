// CPU check of the plugin's mjModel / mjData lifecycle (csrc/plugin/src/mj_types.cpp), built and
// run by tests/test_plugin.py::test_mj_types_lifecycle.  argv[1] = an MJCF scene.  Prints "ok" or
// the first failed check.
#include <cmath>
#include <cstdio>
#include <cstring>

#include "mujoco_ros2_control/mj_types.hpp"

#define CHECK(c)                                     \
  do {                                               \
    if (!(c)) {                                      \
      std::printf("FAIL line %d: %s\n", __LINE__, #c); \
      return 1;                                      \
    }                                                \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  char err[512];
  mrs_model* h = mrs_model_load_xml(argv[1], err, sizeof err);
  CHECK(h != nullptr);
  mjModel* m = mj_wrapModel(h);
  CHECK(m && m->handle == h && m->nq > 0 && m->opt.timestep == m->timestep);

  // get_model: a fresh deep copy, then a copy into an existing mjModel
  mjModel* c = nullptr;
  c = mj_copyModel(c, m);
  CHECK(c && c != m && c->handle != m->handle);
  CHECK(c->nq == m->nq && c->nv == m->nv && c->nu == m->nu && c->nsensordata == m->nsensordata);
  CHECK(c->jnt_qposadr != m->jnt_qposadr);
  for (int j = 0; j < m->njnt; ++j) CHECK(c->jnt_qposadr[j] == m->jnt_qposadr[j]);
  for (int i = 0; i < m->nq; ++i) CHECK(c->qpos0[i] == m->qpos0[i]);
  for (int k = 0; k < 3; ++k) CHECK(c->opt.gravity[k] == m->opt.gravity[k]);
  CHECK(c->opt.solver == m->opt.solver && c->opt.iterations == m->opt.iterations);
  CHECK(mj_copyModel(c, m) == c && c->nbody == m->nbody);
  // the copy outlives its source (mj_copyModel semantics)
  const int nq = m->nq;
  const double q0 = m->qpos0[0];
  mj_deleteModel(m);
  CHECK(c->nq == nq && c->qpos0[0] == q0);

  // get_data / set_data: make, fill, copy into fresh and existing
  mjData* d = mj_makeData(c);
  CHECK(d && d->nq == c->nq && d->time == 0);
  for (int i = 0; i < c->nq; ++i) CHECK(d->qpos[i] == 0);
  for (int i = 0; i < c->nq; ++i) d->qpos[i] = 0.5 + i;
  for (int i = 0; i < c->nv; ++i) d->qvel[i] = -1.0 - i, d->qacc_warmstart[i] = 3.0 * i, d->qfrc_applied[i] = 7;
  for (int i = 0; i < c->nu; ++i) d->ctrl[i] = 0.25 * i;
  for (int i = 0; i < c->nsensordata; ++i) d->sensordata[i] = 11.0 + i;
  d->time = 1.25;
  mjData* e = nullptr;
  e = mj_copyData(e, c, d);
  CHECK(e && e != d && e->qpos != d->qpos && e->time == 1.25);
  for (int i = 0; i < c->nq; ++i) CHECK(e->qpos[i] == d->qpos[i]);
  for (int i = 0; i < c->nv; ++i) CHECK(e->qvel[i] == d->qvel[i] && e->qacc_warmstart[i] == d->qacc_warmstart[i]);
  for (int i = 0; i < c->nu; ++i) CHECK(e->ctrl[i] == d->ctrl[i]);
  for (int i = 0; i < c->nsensordata; ++i) CHECK(e->sensordata[i] == d->sensordata[i]);
  d->time = 2.5;
  d->qpos[0] = -9;
  CHECK(mj_copyData(e, c, d) == e && e->time == 2.5 && e->qpos[0] == -9);

  // a model of another size is refused
  mrs_model* h2 = mrs_model_load_xml_string(
      "<mujoco><worldbody><body><freejoint/><geom size='.1'/></body></worldbody></mujoco>", ".", err, sizeof err);
  CHECK(h2 != nullptr);
  mjModel* m2 = mj_wrapModel(h2);
  if (m2->nq != c->nq) CHECK(mj_copyData(e, m2, d) == nullptr);
  mj_deleteModel(m2);
  mj_deleteData(d);
  mj_deleteData(e);
  mj_deleteModel(c);
  CHECK(mj_wrapModel(nullptr) == nullptr && mj_copyModel(nullptr, nullptr) == nullptr);
  std::printf("ok\n");
  return 0;
}
