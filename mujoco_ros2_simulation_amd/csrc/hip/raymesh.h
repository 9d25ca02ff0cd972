// Ray vs mesh, shared by the step kernel's rangefinders (step.hip) and the depth / colour kernels
// (batch.hip).  mj_rayMesh restated (oracle.c ray_mesh): the ray in the geom frame (origin lp,
// direction lv) is first tested against the geom's bounding box (half extents s, slab test), then
// against the triangles, both faces (Moller-Trumbore) -- the ones the mesh's bounding volume
// hierarchy does not rule out.  `trirec` points at the mesh's first pre-gathered triangle record
// (DevModel::mesh_tri, 9 floats per triangle in device face order).  Returns the nearest t >= 0, or
// -1; *tri gets the nearest triangle when tri is not null.
#pragma once

// Moller-Trumbore core with explicit fmaf chains: the result does not depend on how the compiler
// contracts the surrounding code (the backend fuses multiply-adds freely), so every call site -- the
// every-triangle loop, the hierarchy walk, the binned frame kernel -- gets the same t bit for bit
__device__ __forceinline__ float mt_core(const float a[3], const float e1[3], const float e2[3], const float lp[3],
                                         const float lv[3]) {
  const float pv[3] = {fmaf(lv[1], e2[2], -(lv[2] * e2[1])), fmaf(lv[2], e2[0], -(lv[0] * e2[2])),
                       fmaf(lv[0], e2[1], -(lv[1] * e2[0]))};
  const float det = fmaf(e1[0], pv[0], fmaf(e1[1], pv[1], e1[2] * pv[2]));
  if (fabsf(det) < 1e-15f) return -1;
  const float inv = 1.0f / det;
  const float tv[3] = {lp[0] - a[0], lp[1] - a[1], lp[2] - a[2]};
  const float u = fmaf(tv[0], pv[0], fmaf(tv[1], pv[1], tv[2] * pv[2])) * inv;
  if (u < 0 || u > 1) return -1;
  const float qv[3] = {fmaf(tv[1], e1[2], -(tv[2] * e1[1])), fmaf(tv[2], e1[0], -(tv[0] * e1[2])),
                       fmaf(tv[0], e1[1], -(tv[1] * e1[0]))};
  const float v = fmaf(lv[0], qv[0], fmaf(lv[1], qv[1], lv[2] * qv[2])) * inv;
  if (v < 0 || u + v > 1) return -1;
  const float t = fmaf(e2[0], qv[0], fmaf(e2[1], qv[1], e2[2] * qv[2])) * inv;
  return t >= 0 ? t : -1;
}

// one triangle, both faces (Moller-Trumbore); t >= 0 of the hit or -1
template <class PV, class PF>
__device__ __forceinline__ float ray_tri(PV vert, PF face, int f, const float lp[3], const float lv[3]) {
  const int ia = 3 * face[3 * f], ib = 3 * face[3 * f + 1], ic = 3 * face[3 * f + 2];
  const float a[3] = {vert[ia], vert[ia + 1], vert[ia + 2]};
  const float e1[3] = {vert[ib] - a[0], vert[ib + 1] - a[1], vert[ib + 2] - a[2]};
  const float e2[3] = {vert[ic] - a[0], vert[ic + 1] - a[1], vert[ic + 2] - a[2]};
  return mt_core(a, e1, e2, lp, lv);
}

// a pixel ray (camera-frame slopes dx, dy; direction (dx, dy, -1)) in a geom frame: rows of A
template <class PA>
__device__ __forceinline__ void pixel_ray(const PA A, float dx, float dy, float lv[3]) {
  lv[0] = fmaf(A[0], dx, fmaf(A[1], dy, -A[2]));
  lv[1] = fmaf(A[3], dx, fmaf(A[4], dy, -A[5]));
  lv[2] = fmaf(A[6], dx, fmaf(A[7], dy, -A[8]));
}

// one pre-gathered triangle record (vertex a, edges e1 = b - a, e2 = c - a: DevModel::mesh_tri), both
// faces; the expressions of ray_tri in the same order, so t is bit-identical to it
template <class PT>
__device__ __forceinline__ float ray_tri_rec(PT tri, int f, const float lp[3], const float lv[3]) {
  const int o = 9 * f;
  const float a[3] = {tri[o], tri[o + 1], tri[o + 2]};
  const float e1[3] = {tri[o + 3], tri[o + 4], tri[o + 5]};
  const float e2[3] = {tri[o + 6], tri[o + 7], tri[o + 8]};
  return mt_core(a, e1, e2, lp, lv);
}

// slab test of the ray against an axis-aligned box [lo, hi]: the entry parameter, or 3e38 on a miss
__device__ __forceinline__ float ray_aabb(const float lo[3], const float hi[3], const float lp[3], const float lv[3],
                                          const float iv[3]) {
  float tmin = -3.0e38f, tmax = 3.0e38f;
  for (int i = 0; i < 3; ++i) {
    if (fabsf(lv[i]) < 1e-15f) {
      if (lp[i] < lo[i] || lp[i] > hi[i]) return 3.0e38f;
      continue;
    }
    const float t1 = (lo[i] - lp[i]) * iv[i], t2 = (hi[i] - lp[i]) * iv[i];
    tmin = fmaxf(tmin, fminf(t1, t2));
    tmax = fminf(tmax, fmaxf(t1, t2));
  }
  return (tmax < tmin || tmax < 0) ? 3.0e38f : tmin;
}

// The nearest hit over the triangles is the same whichever triangles the bounding volumes let
// through (each triangle's t is computed by ray_tri alike); only ties between triangles at equal t
// may resolve to a different triangle (its normal shades the colour image).
// bvh / nnode: the mesh's bounding volume hierarchy (batch.hip build_mesh_bvh): 8 floats per node in
// depth-first order -- AABB lo, the index of the node after its subtree (int bits), AABB hi, and for a
// leaf (first << 8 | count) of its triangles in `face` (int bits; -1 for an inner node).  Stackless
// traversal per lane: a missed box, a box entered past the nearest hit, or a leaf jumps to the skip
// index, an inner node that is hit descends to its first child (the next node); both successors are
// loaded while a node is tested, so a step costs one memory latency.  nnode = 0: every triangle.
// (A wave-coherent packet walk -- node index by ballot, scalar loads -- measured slower at both call
// sites on the mesh robot: step 26.7 vs 12.8 ms, depth 501 vs 442 ms: the union of 64 rays' paths
// visits far more nodes than one ray's.)
// bound >= 0: a hit already known along the ray (the caller's nearest so far); only nearer triangles
// count, boxes entered beyond it are skipped (a ray through a closed shell whose inside hit is known
// never walks the far side), and the result is bound itself when nothing nearer is found
template <class PT, class PS, class PN>
__device__ __forceinline__ float ray_mesh(PT trirec, int nface, const PS s, const float lp[3],
                                          const float lv[3], PN bvh, int nnode, int* tri = nullptr,
                                          float bound = -1.0f) {
  {
    const float lo[3] = {-s[0], -s[1], -s[2]}, hi[3] = {s[0], s[1], s[2]};
    const float iv[3] = {1.0f / lv[0], 1.0f / lv[1], 1.0f / lv[2]};
    const float te = ray_aabb(lo, hi, lp, lv, iv);
    if (te == 3.0e38f || (bound >= 0 && te > bound)) return -1;
  }
  float best = bound;
  if (nnode <= 0) {
    for (int f = 0; f < nface; ++f) {
      const float t = ray_tri_rec(trirec, f, lp, lv);
      if (t >= 0 && (best < 0 || t < best)) { best = t; if (tri) *tri = f; }
    }
    return best;
  }
  const float iv[3] = {1.0f / lv[0], 1.0f / lv[1], 1.0f / lv[2]};
  struct Node { float lo[3], hi[3]; int skip, leaf; };
  auto load = [&](int k) {
    const int o = 8 * k;
    Node n;
    n.lo[0] = bvh[o]; n.lo[1] = bvh[o + 1]; n.lo[2] = bvh[o + 2]; n.skip = __float_as_int(bvh[o + 3]);
    n.hi[0] = bvh[o + 4]; n.hi[1] = bvh[o + 5]; n.hi[2] = bvh[o + 6]; n.leaf = __float_as_int(bvh[o + 7]);
    return n;
  };
  int i = 0;
  Node cur = load(0);
  while (i < nnode) {
    const Node down = load(i + 1 < nnode ? i + 1 : i);
    const Node side = load(cur.skip < nnode ? cur.skip : i);
    const float te = ray_aabb(cur.lo, cur.hi, lp, lv, iv);
    const bool hit = te != 3.0e38f && (best < 0 || te <= best);
    if (hit && cur.leaf >= 0) {
      const int f0 = cur.leaf >> 8, nf = cur.leaf & 0xff;
      for (int f = f0; f < f0 + nf; ++f) {
        const float t = ray_tri_rec(trirec, f, lp, lv);
        if (t >= 0 && (best < 0 || t < best)) { best = t; if (tri) *tri = f; }
      }
    }
    const bool descend = hit && cur.leaf < 0;
    i = descend ? i + 1 : cur.skip;
    cur = descend ? down : side;
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
