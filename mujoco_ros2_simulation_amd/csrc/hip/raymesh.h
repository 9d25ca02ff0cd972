// Ray vs mesh, shared by the step kernel's rangefinders (step.hip) and the depth / colour kernels
// (batch.hip).  mj_rayMesh restated (oracle.c ray_mesh): the ray in the geom frame (origin lp,
// direction lv) is first tested against the geom's bounding box (half extents s, slab test), then
// against every triangle, both faces (Moller-Trumbore).  `vert` / `face` point at the mesh's own
// vertices and triangles (face ids relative to vert).  Returns the nearest t >= 0, or -1; *tri gets
// the nearest triangle when tri is not null.
#pragma once

template <class PV, class PF, class PS>
__device__ __forceinline__ float ray_mesh(PV vert, PF face, int nface, const PS s, const float lp[3],
                                          const float lv[3], int* tri = nullptr) {
  float tmin = -3.0e38f, tmax = 3.0e38f;
  for (int i = 0; i < 3; ++i) {
    if (fabsf(lv[i]) < 1e-15f) {
      if (fabsf(lp[i]) > s[i]) return -1;
      continue;
    }
    const float t1 = (-s[i] - lp[i]) / lv[i], t2 = (s[i] - lp[i]) / lv[i];
    tmin = fmaxf(tmin, fminf(t1, t2));
    tmax = fminf(tmax, fmaxf(t1, t2));
  }
  if (tmax < tmin || tmax < 0) return -1;
  float best = -1;
  for (int f = 0; f < nface; ++f) {
    const int ia = 3 * face[3 * f], ib = 3 * face[3 * f + 1], ic = 3 * face[3 * f + 2];
    const float a[3] = {vert[ia], vert[ia + 1], vert[ia + 2]};
    const float e1[3] = {vert[ib] - a[0], vert[ib + 1] - a[1], vert[ib + 2] - a[2]};
    const float e2[3] = {vert[ic] - a[0], vert[ic + 1] - a[1], vert[ic + 2] - a[2]};
    const float pv[3] = {lv[1] * e2[2] - lv[2] * e2[1], lv[2] * e2[0] - lv[0] * e2[2], lv[0] * e2[1] - lv[1] * e2[0]};
    const float det = e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2];
    if (fabsf(det) < 1e-15f) continue;
    const float inv = 1.0f / det;
    const float tv[3] = {lp[0] - a[0], lp[1] - a[1], lp[2] - a[2]};
    const float u = (tv[0] * pv[0] + tv[1] * pv[1] + tv[2] * pv[2]) * inv;
    if (u < 0 || u > 1) continue;
    const float qv[3] = {tv[1] * e1[2] - tv[2] * e1[1], tv[2] * e1[0] - tv[0] * e1[2], tv[0] * e1[1] - tv[1] * e1[0]};
    const float v = (lv[0] * qv[0] + lv[1] * qv[1] + lv[2] * qv[2]) * inv;
    if (v < 0 || u + v > 1) continue;
    const float t = (e2[0] * qv[0] + e2[1] * qv[1] + e2[2] * qv[2]) * inv;
    if (t >= 0 && (best < 0 || t < best)) {
      best = t;
      if (tri) *tri = f;
    }
  }
  return best;
}

// unnormalised normal of triangle f of a mesh, turned to face against the ray direction lv (two-sided)
template <class PV, class PF>
__device__ __forceinline__ void mesh_tri_normal(PV vert, PF face, int f, const float lv[3], float n[3]) {
  const int ia = 3 * face[3 * f], ib = 3 * face[3 * f + 1], ic = 3 * face[3 * f + 2];
  const float e1[3] = {vert[ib] - vert[ia], vert[ib + 1] - vert[ia + 1], vert[ib + 2] - vert[ia + 2]};
  const float e2[3] = {vert[ic] - vert[ia], vert[ic + 1] - vert[ia + 1], vert[ic + 2] - vert[ia + 2]};
  n[0] = e1[1] * e2[2] - e1[2] * e2[1];
  n[1] = e1[2] * e2[0] - e1[0] * e2[2];
  n[2] = e1[0] * e2[1] - e1[1] * e2[0];
  if (n[0] * lv[0] + n[1] * lv[1] + n[2] * lv[2] > 0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
}
