// mjModel / mjData lifecycle (include/mujoco_ros2_control/mj_types.hpp).
#include "mujoco_ros2_control/mj_types.hpp"

#include <cstring>
#include <new>

namespace {

void fill_view(mjModel* m) {
  mrs_model_view v{};
  mrs_model_view_get(m->handle, &v);
  static_cast<mrs_model_view&>(*m) = v;
  mjOption& o = m->opt;
  o.timestep = v.timestep;
  for (int k = 0; k < 3; ++k) o.gravity[k] = v.gravity[k];
  o.tolerance = v.tolerance;
  o.impratio = v.impratio;
  o.ls_tolerance = v.ls_tolerance;
  o.integrator = v.integrator;
  o.solver = v.solver;
  o.iterations = v.iterations;
  o.ls_iterations = v.ls_iterations;
  o.cone = v.cone;
  o.disableflags = v.disableflags;
}

}  // namespace

mjModel* mj_wrapModel(mrs_model* handle) {
  if (!handle) return nullptr;
  mjModel* m = new mjModel();
  m->handle = handle;
  fill_view(m);
  return m;
}

mjModel* mj_copyModel(mjModel* dest, const mjModel* src) {
  if (!src || !src->handle) return nullptr;
  mrs_model* copy = mrs_model_copy(src->handle);
  if (!copy) return nullptr;
  if (!dest) return mj_wrapModel(copy);
  mrs_model_free(dest->handle);
  dest->handle = copy;
  fill_view(dest);
  return dest;
}

void mj_deleteModel(mjModel* m) {
  if (!m) return;
  mrs_model_free(m->handle);
  delete m;
}

mjData* mj_makeData(const mjModel* m) {
  if (!m) return nullptr;
  mjData* d = new mjData();
  d->nq = m->nq;
  d->nv = m->nv;
  d->nu = m->nu;
  d->nsensordata = m->nsensordata;
  const size_t n = size_t(d->nq) + 5 * size_t(d->nv) + size_t(d->nu) + size_t(d->nsensordata);
  d->buffer = new double[n > 0 ? n : 1]();
  double* p = d->buffer;
  auto take = [&p](int k) { double* r = p; p += k; return r; };
  d->qpos = take(d->nq);
  d->qvel = take(d->nv);
  d->qacc = take(d->nv);
  d->qacc_warmstart = take(d->nv);
  d->ctrl = take(d->nu);
  d->qfrc_applied = take(d->nv);
  d->qfrc_actuator = take(d->nv);
  d->sensordata = take(d->nsensordata);
  return d;
}

mjData* mj_copyData(mjData* dest, const mjModel* m, const mjData* src) {
  if (!m || !src) return nullptr;
  if (src->nq != m->nq || src->nv != m->nv || src->nu != m->nu || src->nsensordata != m->nsensordata)
    return nullptr;
  if (!dest) dest = mj_makeData(m);
  else if (dest->nq != m->nq || dest->nv != m->nv || dest->nu != m->nu || dest->nsensordata != m->nsensordata)
    return nullptr;
  const size_t n = size_t(m->nq) + 5 * size_t(m->nv) + size_t(m->nu) + size_t(m->nsensordata);
  if (dest != src) std::memcpy(dest->buffer, src->buffer, n * sizeof(double));
  dest->time = src->time;
  return dest;
}

void mj_deleteData(mjData* d) {
  if (!d) return;
  delete[] d->buffer;
  delete d;
}
