// Batch of environments resident on one GPU: model packing, memory layouts, state transfer,
// step/forward launches and the depth-camera kernel.  Host side of the C ABI in include/mrs.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/mrs.h"
#include "../mjcf/model.h"
#include "batch.h"
#include "devmodel.h"
#include "raymesh.h"
#include "lit.h"

namespace mrs {

hipError_t launch_step(const DevModel* d_model, int lds_floats, int shared_floats, const DevState& st, int n_envs,
                       int n_steps, bool forward_only, int group, bool primal, bool ext, hipStream_t stream);

namespace {

#define HIP_CHECK(x)                                                                         \
  do {                                                                                       \
    hipError_t err_ = (x);                                                                   \
    if (err_ != hipSuccess)                                                                  \
      throw DeviceError(std::string(#x) + " failed: " + hipGetErrorString(err_));            \
  } while (0)

// ------------------------------------------------------------------ depth camera kernel
// One thread per pixel, one env per blockIdx.y; the env's geom poses are staged in LDS.
// Eye-space depth: ray through the pixel centre with camera-frame direction (x, y, -1), so the ray
// parameter of the nearest hit is the eye-space z that OpenGL + the plugin's linearisation
// (src/mujoco_cameras.cpp:222-235) produce; rows in ROS order (flip of :229-240 applied).
constexpr int kMaxRenderGeoms = 256;
// the model's meshes for the render kernels (mrs_model.h mesh arrays, device copies)
struct MeshRef {
  const float* vert;
  const int *face, *dataid, *vertadr, *faceadr, *facenum;
  const float* bvh;           // bounding volume hierarchies (8 floats per node, build_mesh_bvh)
  const int *bvhadr, *bvhnum;  // per mesh: first node, node count (0: no hierarchy, every triangle)
  const float* tri;            // pre-gathered triangle records (DevModel::mesh_tri)
};

// analytic ray primitive (same restatement of engine_ray as the step kernel's rangefinder)
__device__ float ray_prim(int type, const float* s, const float lp[3], const float lv[3]) {
  auto quad = [](float a, float b, float c, float x[2]) {
    float det = b * b - a * c;
    if (det < 1e-15f) { x[0] = x[1] = -1; return -1.0f; }
    det = sqrtf(det);
    x[0] = (-b - det) / a;
    x[1] = (-b + det) / a;
    if (x[0] >= 0) return x[0];
    if (x[1] >= 0) return x[1];
    return -1.0f;
  };
  auto d3 = [](const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
  float x[2];
  switch (type) {
    case MRS_GEOM_PLANE: {
      if (lv[2] >= 0 || lv[2] * lv[2] <= 1e-12f * d3(lv, lv)) return -1;
      float t = -lp[2] / lv[2];
      if (t < 0) return -1;
      float p0 = lp[0] + t * lv[0], p1 = lp[1] + t * lv[1];
      if ((s[0] <= 0 || fabsf(p0) <= s[0]) && (s[1] <= 0 || fabsf(p1) <= s[1])) return t;
      return -1;
    }
    case MRS_GEOM_SPHERE: return quad(d3(lv, lv), d3(lv, lp), d3(lp, lp) - s[0] * s[0], x);
    case MRS_GEOM_CAPSULE: {
      float best = -1;
      float a = lv[0] * lv[0] + lv[1] * lv[1];
      if (a > 1e-15f) {
        quad(a, lv[0] * lp[0] + lv[1] * lp[1], lp[0] * lp[0] + lp[1] * lp[1] - s[0] * s[0], x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && fabsf(lp[2] + x[i] * lv[2]) <= s[1] && (best < 0 || x[i] < best)) best = x[i];
      }
      for (int e = -1; e <= 1; e += 2) {
        float q[3] = {lp[0], lp[1], lp[2] - e * s[1]};
        quad(d3(lv, lv), d3(lv, q), d3(q, q) - s[0] * s[0], x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && e * (lp[2] + x[i] * lv[2] - e * s[1]) >= 0 && (best < 0 || x[i] < best)) best = x[i];
      }
      return best;
    }
    case MRS_GEOM_ELLIPSOID: {
      float q[3] = {lp[0] / s[0], lp[1] / s[1], lp[2] / s[2]}, v[3] = {lv[0] / s[0], lv[1] / s[1], lv[2] / s[2]};
      return quad(d3(v, v), d3(v, q), d3(q, q) - 1, x);
    }
    case MRS_GEOM_CYLINDER: {
      float best = -1;
      float a = lv[0] * lv[0] + lv[1] * lv[1];
      if (a > 1e-15f) {
        quad(a, lv[0] * lp[0] + lv[1] * lp[1], lp[0] * lp[0] + lp[1] * lp[1] - s[0] * s[0], x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && fabsf(lp[2] + x[i] * lv[2]) <= s[1] && (best < 0 || x[i] < best)) best = x[i];
      }
      if (fabsf(lv[2]) > 1e-15f)
        for (int e = -1; e <= 1; e += 2) {
          float t = (e * s[1] - lp[2]) / lv[2];
          if (t < 0) continue;
          float p0 = lp[0] + t * lv[0], p1 = lp[1] + t * lv[1];
          if (p0 * p0 + p1 * p1 <= s[0] * s[0] && (best < 0 || t < best)) best = t;
        }
      return best;
    }
    case MRS_GEOM_BOX: {
      float best = -1;
      for (int i = 0; i < 3; ++i) {
        if (fabsf(lv[i]) <= 1e-15f) continue;
        int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
        for (int side = -1; side <= 1; side += 2) {
          float t = (side * s[i] - lp[i]) / lv[i];
          if (t < 0) continue;
          float p1 = lp[i1] + t * lv[i1], p2 = lp[i2] + t * lv[i2];
          if (fabsf(p1) <= s[i1] && fabsf(p2) <= s[i2] && (best < 0 || t < best)) best = t;
        }
      }
      return best;
    }
  }
  return -1;
}


// ---- colour: the lit model of lit.h (oracle.c lit_color restates it in fp64); local_normal gives
// the geom-frame surface normal (unnormalised) at a hit point p
__device__ __forceinline__ void local_normal(int type, const float* s, const float p[3], float n[3]) {
  n[0] = 0; n[1] = 0; n[2] = 1;
  switch (type) {
    case MRS_GEOM_SPHERE: n[0] = p[0]; n[1] = p[1]; n[2] = p[2]; break;
    case MRS_GEOM_CAPSULE: n[0] = p[0]; n[1] = p[1]; n[2] = p[2] - fminf(fmaxf(p[2], -s[1]), s[1]); break;
    case MRS_GEOM_ELLIPSOID: n[0] = p[0] / (s[0] * s[0]); n[1] = p[1] / (s[1] * s[1]); n[2] = p[2] / (s[2] * s[2]); break;
    case MRS_GEOM_CYLINDER: {
      const float rr = sqrtf(p[0] * p[0] + p[1] * p[1]);
      if (fabsf(p[2]) - s[1] > rr - s[0]) { n[0] = 0; n[1] = 0; n[2] = p[2] >= 0 ? 1.0f : -1.0f; }
      else { n[0] = p[0]; n[1] = p[1]; n[2] = 0; }
      break;
    }
    case MRS_GEOM_BOX: {
      int k = 0;
      float best = fabsf(p[0]) / s[0];
      for (int i = 1; i < 3; ++i)
        if (fabsf(p[i]) / s[i] > best) { best = fabsf(p[i]) / s[i]; k = i; }
      n[0] = 0; n[1] = 0; n[2] = 0;
      n[k] = p[k] >= 0 ? 1.0f : -1.0f;
      break;
    }
    default: break;
  }
}

// One workgroup renders a 16x16-pixel tile of one env.  The tile's pixel rays lie inside a cone
// (apex at the camera, axis through the tile centre, half-angle to the widest corner ray); a geom
// whose bounding sphere misses that cone, or a plane no ray of the cone can reach, is skipped by the
// whole tile, and the pixels test only the remaining candidates.  Culling only removes geoms no pixel
// ray can hit, so every pixel keeps the nearest hit over all geoms.
template <bool kRGB>
__global__ __launch_bounds__(256) void depth_kernel(const int* geom_type, const int* geom_group,
                                                    const float* geom_size, const float* geom_rbound,
                                                    const float* geom_rgba, int ngeom, const float* geom_xpos,
                                                    const float* geom_xmat, const float* cam_xpos,
                                                    const float* cam_xmat, int ncam, int cam, int env0, int W,
                                                    int H, float f, float znear, float zfar, float* out,
                                                    unsigned char* rgb, MeshRef mesh, LitRef lr) {
  __shared__ float gp[kMaxRenderGeoms * 3];
  __shared__ LitFrame LF;
  __shared__ float gm[kMaxRenderGeoms * 9];
  __shared__ float cpos[3], cmat[9];
  __shared__ int cand[kMaxRenderGeoms];
  __shared__ int ncand;
  const int env = env0 + blockIdx.y;
  const size_t eo = (size_t)env;
  for (int i = threadIdx.x; i < 3 * ngeom; i += blockDim.x) gp[i] = geom_xpos[eo * 3 * ngeom + i];
  for (int i = threadIdx.x; i < 9 * ngeom; i += blockDim.x) gm[i] = geom_xmat[eo * 9 * ngeom + i];
  if (threadIdx.x < 3) cpos[threadIdx.x] = cam_xpos[(eo * ncam + cam) * 3 + threadIdx.x];
  if (threadIdx.x < 9) cmat[threadIdx.x] = cam_xmat[(eo * ncam + cam) * 9 + threadIdx.x];
  if (threadIdx.x == 0) ncand = 0;
  if (kRGB && threadIdx.x == 255)
    lit_stage(LF, lr, cam_xpos + (eo * ncam + cam) * 3, cam_xmat + (eo * ncam + cam) * 9);
  const int tiles_x = (W + 15) / 16;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
  __syncthreads();
  if (threadIdx.x < ngeom) {
    const int g = threadIdx.x;
    const int grp = geom_group[g];
    bool keep = !(grp < 0 || grp > 2 || geom_rgba[4 * g + 3] == 0);
    if (keep) {
      // tile cone in the camera frame, then world: axis through the tile centre, cos of the widest
      // corner angle (pixel centres of the tile's extreme rows/columns)
      const float c0 = tx * 16 + 0.5f, c1 = fminf(tx * 16 + 15.0f, W - 1.0f) + 0.5f;
      const float r0 = ty * 16 + 0.5f, r1 = fminf(ty * 16 + 15.0f, H - 1.0f) + 0.5f;
      float ac[3] = {(0.5f * (c0 + c1) - 0.5f * W) / f, (0.5f * H - 0.5f * (r0 + r1)) / f, -1.0f};
      const float an = sqrtf(ac[0] * ac[0] + ac[1] * ac[1] + 1.0f);
      ac[0] /= an; ac[1] /= an; ac[2] /= an;
      float cth = 1.0f;
      for (int k = 0; k < 4; ++k) {
        const float cc = (k & 1) ? c1 : c0, rr = (k & 2) ? r1 : r0;
        const float dx = (cc - 0.5f * W) / f, dy = (0.5f * H - rr) / f;
        const float dn = sqrtf(dx * dx + dy * dy + 1.0f);
        cth = fminf(cth, (dx * ac[0] + dy * ac[1] - ac[2]) / dn);
      }
      cth = fmaxf(-1.0f, cth - 1e-4f);
      const float sth = sqrtf(fmaxf(0.0f, 1.0f - cth * cth));
      const float a[3] = {cmat[0] * ac[0] + cmat[1] * ac[1] + cmat[2] * ac[2],
                          cmat[3] * ac[0] + cmat[4] * ac[1] + cmat[5] * ac[2],
                          cmat[6] * ac[0] + cmat[7] * ac[1] + cmat[8] * ac[2]};
      const float v[3] = {gp[3 * g] - cpos[0], gp[3 * g + 1] - cpos[1], gp[3 * g + 2] - cpos[2]};
      if (geom_type[g] == MRS_GEOM_PLANE) {
        // origin in front of the plane and some direction of the cone with d.n < 0:
        // min over the cone of d.n = cos(angle(a, n) + theta)
        const float n[3] = {gm[9 * g + 2], gm[9 * g + 5], gm[9 * g + 8]};
        const float an2 = a[0] * n[0] + a[1] * n[1] + a[2] * n[2];
        const float mind = an2 * cth - sqrtf(fmaxf(0.0f, 1.0f - an2 * an2)) * sth;
        keep = -(v[0] * n[0] + v[1] * n[1] + v[2] * n[2]) > 0 && mind < 1e-6f;
      } else {
        const float rb = geom_rbound[g] * 1.001f + 1e-4f;
        const float l2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        if (l2 > rb * rb) {
          // angle(v, a) <= theta + asin(rb/|v|)  <=>  v.a >= |v| cos(theta) cos(beta) - rb sin(theta)
          const float l = sqrtf(l2);
          const float va = v[0] * a[0] + v[1] * a[1] + v[2] * a[2];
          keep = va >= cth * sqrtf(l2 - rb * rb) - sth * rb - 1e-6f * l;
        }
      }
    }
    if (keep) cand[atomicAdd(&ncand, 1)] = g;
  }
  __syncthreads();
  const int row = ty * 16 + threadIdx.x / 16, col = tx * 16 + threadIdx.x % 16;
  if (row >= H || col >= W) return;
  const int pix = row * W + col;
  const float dc[3] = {(col + 0.5f - 0.5f * W) / f, (0.5f * H - row - 0.5f) / f, -1.0f};
  const float vec[3] = {cmat[0] * dc[0] + cmat[1] * dc[1] + cmat[2] * dc[2],
                        cmat[3] * dc[0] + cmat[4] * dc[1] + cmat[5] * dc[2],
                        cmat[6] * dc[0] + cmat[7] * dc[1] + cmat[8] * dc[2]};
  const float vv = vec[0] * vec[0] + vec[1] * vec[1] + vec[2] * vec[2];
  float best = -1;
  int bestg = -1;
  const int nc = ncand;
  for (int i = 0; i < nc; ++i) {
    const int g = cand[i];
    const float* p = gp + 3 * g;
    const float* mm = gm + 9 * g;
    const float dv[3] = {cpos[0] - p[0], cpos[1] - p[1], cpos[2] - p[2]};
    const int t = geom_type[g];
    if (t != MRS_GEOM_PLANE) {
      // bounding-sphere reject: closest approach of the ray to the geom centre
      const float dvv = dv[0] * vec[0] + dv[1] * vec[1] + dv[2] * vec[2];
      const float dd = dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2];
      const float rb = geom_rbound[g];
      if (dd - dvv * dvv / vv > rb * rb) continue;
    }
    const float lp[3] = {mm[0] * dv[0] + mm[3] * dv[1] + mm[6] * dv[2], mm[1] * dv[0] + mm[4] * dv[1] + mm[7] * dv[2],
                         mm[2] * dv[0] + mm[5] * dv[1] + mm[8] * dv[2]};
    const float lv[3] = {mm[0] * vec[0] + mm[3] * vec[1] + mm[6] * vec[2],
                         mm[1] * vec[0] + mm[4] * vec[1] + mm[7] * vec[2],
                         mm[2] * vec[0] + mm[5] * vec[1] + mm[8] * vec[2]};
    float tt;
    if (t == MRS_GEOM_MESH) {
      const int id = mesh.dataid[g];
      int tri;
      tt = ray_mesh(mesh.tri + 9 * mesh.faceadr[id], mesh.facenum[id], geom_size + 3 * g, lp, lv,
                    mesh.bvh + 8 * mesh.bvhadr[id], mesh.bvhnum[id], &tri);
    } else {
      tt = ray_prim(t, geom_size + 3 * g, lp, lv);
    }
    if (tt >= znear && (best < 0 || tt < best)) { best = tt; bestg = g; }
  }
  const bool hit = !(best < 0 || best > zfar);
  out[(size_t)blockIdx.y * W * H + pix] = hit ? best : zfar;
  if constexpr (kRGB) {
    unsigned char* px = rgb + ((size_t)blockIdx.y * W * H + pix) * 3;
    if (!hit) { lit_sky(LF, dc[0], dc[1], px); return; }
    const float* p = gp + 3 * bestg;
    const float* mm = gm + 9 * bestg;
    const float dv[3] = {cpos[0] - p[0], cpos[1] - p[1], cpos[2] - p[2]};
    float q[3], nl[3], nw[3], nc[3];
    for (int i = 0; i < 3; ++i)
      q[i] = mm[i] * dv[0] + mm[3 + i] * dv[1] + mm[6 + i] * dv[2] +
             best * (mm[i] * vec[0] + mm[3 + i] * vec[1] + mm[6 + i] * vec[2]);
    if (geom_type[bestg] == MRS_GEOM_MESH) {  // the hit triangle's normal, facing the ray
      const int id = mesh.dataid[bestg];
      const float* mv = mesh.vert + 3 * mesh.vertadr[id];
      const int* mf = mesh.face + 3 * mesh.faceadr[id];
      float lp[3], lv[3];
      for (int i = 0; i < 3; ++i) {
        lp[i] = mm[i] * dv[0] + mm[3 + i] * dv[1] + mm[6 + i] * dv[2];
        lv[i] = mm[i] * vec[0] + mm[3 + i] * vec[1] + mm[6 + i] * vec[2];
      }
      int tri = 0;
      ray_mesh(mesh.tri + 9 * mesh.faceadr[id], mesh.facenum[id], geom_size + 3 * bestg, lp, lv,
               mesh.bvh + 8 * mesh.bvhadr[id], mesh.bvhnum[id], &tri);
      mesh_tri_normal(mv, mf, tri, lv, nl);
    } else {
      local_normal(geom_type[bestg], geom_size + 3 * bestg, q, nl);
    }
    for (int i = 0; i < 3; ++i) nw[i] = mm[3 * i] * nl[0] + mm[3 * i + 1] * nl[1] + mm[3 * i + 2] * nl[2];
    for (int j = 0; j < 3; ++j) nc[j] = cmat[j] * nw[0] + cmat[3 + j] * nw[1] + cmat[6 + j] * nw[2];
    float rgba3[3] = {geom_rgba[4 * bestg], geom_rgba[4 * bestg + 1], geom_rgba[4 * bestg + 2]};
    // shadow rays in the world frame: every geom of groups 0-2 with alpha > 0, bounding-sphere reject
    auto occ = [&](const float* o, const float* L, float dist) {
      float ow[3], lw[3];
      for (int i = 0; i < 3; ++i) {
        ow[i] = cpos[i] + cmat[3 * i] * o[0] + cmat[3 * i + 1] * o[1] + cmat[3 * i + 2] * o[2];
        lw[i] = cmat[3 * i] * L[0] + cmat[3 * i + 1] * L[1] + cmat[3 * i + 2] * L[2];
      }
      for (int g = 0; g < ngeom; ++g) {
        const int grp = geom_group[g];
        if (grp < 0 || grp > 2 || geom_rgba[4 * g + 3] == 0) continue;
        const float* gpp = gp + 3 * g;
        const float* gmm = gm + 9 * g;
        const float d[3] = {ow[0] - gpp[0], ow[1] - gpp[1], ow[2] - gpp[2]};
        const int t = geom_type[g];
        if (t != MRS_GEOM_PLANE) {
          const float rb = geom_rbound[g] * 1.001f + 1e-4f;
          const float pr = -(d[0] * lw[0] + d[1] * lw[1] + d[2] * lw[2]);
          const float dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
          if (dd > rb * rb && (pr < 0 || dd - pr * pr > rb * rb)) continue;
        }
        float lp[3], lv[3];
        for (int i = 0; i < 3; ++i) {
          lp[i] = gmm[i] * d[0] + gmm[3 + i] * d[1] + gmm[6 + i] * d[2];
          lv[i] = gmm[i] * lw[0] + gmm[3 + i] * lw[1] + gmm[6 + i] * lw[2];
        }
        float th;
        if (t == MRS_GEOM_MESH) {
          const int id = mesh.dataid[g];
          int tri;
          th = ray_mesh(mesh.tri + 9 * mesh.faceadr[id], mesh.facenum[id], geom_size + 3 * g, lp, lv,
                        mesh.bvh + 8 * mesh.bvhadr[id], mesh.bvhnum[id], &tri);
        } else {
          th = ray_prim(t, geom_size + 3 * g, lp, lv);
        }
        if (th >= 0 && th < dist) return true;
      }
      return false;
    };
    lit_pixel(LF, lr, bestg, rgba3, geom_type[bestg], geom_size + 3 * bestg, q, dc[0], dc[1], best, nc, occ, px);
  }
}

// ---- depth kernel v2 (ngeom <= 64): one workgroup renders a whole frame of one env.  The
// workgroup stages, once per frame, each visible geom's data in LDS: the camera origin in the geom
// frame lp = R'(c - p) and A = R' C (C: camera rotation), so the geom-frame direction of the pixel
// ray (x, y, -1) is lv = A (x, y, -1) -- three FMAs per component per pixel -- and, for the cull,
// the geom's centre and axes in the camera frame with the half extents of an oriented box around it.
// Each wave walks tiles of 64 x 16 pixels: lane = column (every store is 256 contiguous bytes), 16 rows
// per lane.  Per tile, lane g tests geom g against the tile's pyramid of rays (four planes through
// the camera): an oriented box wholly outside one plane, or a plane no corner ray descends onto, is
// skipped; one ballot gives the candidates and the pixel loop visits only those (wave-uniform geom,
// so the primitive test does not diverge by type).  Boxes use the slab test: the same face
// parameters (+-s - lp) / lv as the face-by-face test, nearest non-negative crossing.
#ifndef MRS_DEPTH_TILE_H
#define MRS_DEPTH_TILE_H 16  // measured C4 (2048 frames): 4 rows 2.08 ms, 8 rows 1.70, 16 rows 1.68, 32 rows 2.13
#endif
#ifndef MRS_DEPTH_CHUNK
#define MRS_DEPTH_CHUNK 8  // rows of a tile evaluated together (registers: the chunk's rows only; measured C4 frames alone 1.66 ms at 8, 1.77 at 4 and 16)
#endif
constexpr int kDepthTileW = 64, kDepthTileH = MRS_DEPTH_TILE_H, kDepthGeoms = 64, kDepthChunk = MRS_DEPTH_CHUNK;
static_assert(kDepthTileH % kDepthChunk == 0, "a tile is a whole number of row chunks");
struct DepthGeom {  // 30 words in LDS
  float lp[3], A[9], size[3];  // row i of A = R'C is also the geom's axis i in the camera frame
  float cc[3], ext[3];         // cull: centre in the camera frame, oriented-box half extents
  float rgba[3];               // colour (RGB output)
  int type, vis, dataid;
  int cast;                    // casts shadows (groups 0-2, alpha > 0; no frustum cull)
};
__device__ __forceinline__ float ray_box_slab(const float* s, const float lp[3], const float lv[3]) {
  float tmin = -3.0e38f, tmax = 3.0e38f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float inv = __builtin_amdgcn_rcpf(lv[i]);
    const bool par = fabsf(lv[i]) <= 1e-15f;
    const float t1 = (-s[i] - lp[i]) * inv, t2 = (s[i] - lp[i]) * inv;
    // a ray parallel to a slab is inside it for all t or for none
    const bool inside = fabsf(lp[i]) <= s[i];
    const float lo = par ? (inside ? -3.0e38f : 3.0e38f) : fminf(t1, t2);
    const float hi = par ? (inside ? 3.0e38f : -3.0e38f) : fmaxf(t1, t2);
    tmin = fmaxf(tmin, lo);
    tmax = fminf(tmax, hi);
  }
  if (tmax < tmin || tmax < 0) return -1;
  return tmin >= 0 ? tmin : tmax;
}
// one visible-geom record of a frame (lane g of the frame's workgroup): the camera origin and the pixel
// ray directions in the geom frame, the geom's culling box in the camera frame, its colour and type
__device__ __forceinline__ void stage_depth_geom(DepthGeom* G, const int* geom_type, const int* geom_group,
                                                 const float* geom_size, const float* geom_rgba, int ngeom,
                                                 const float* geom_xpos, const float* geom_xmat, const float* cp,
                                                 const float* cm, size_t eo, float znear, float zfar, MeshRef mesh) {
  if (threadIdx.x < ngeom) {
    const int g = threadIdx.x;
    const float cpos[3] = {cp[0], cp[1], cp[2]};
    float C[9];
    for (int i = 0; i < 9; ++i) C[i] = cm[i];
    DepthGeom& o = G[g];
    const int grp = geom_group[g];
    o.vis = !(grp < 0 || grp > 2 || geom_rgba[4 * g + 3] == 0);
    o.cast = o.vis;
    const float* p = geom_xpos + eo * 3 * ngeom + 3 * g;
    const float* R = geom_xmat + eo * 9 * ngeom + 9 * g;
    const float d[3] = {cpos[0] - p[0], cpos[1] - p[1], cpos[2] - p[2]};
    for (int i = 0; i < 3; ++i) o.lp[i] = R[i] * d[0] + R[3 + i] * d[1] + R[6 + i] * d[2];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) o.A[3 * i + j] = R[i] * C[j] + R[3 + i] * C[3 + j] + R[6 + i] * C[6 + j];
    for (int i = 0; i < 3; ++i) {
      o.size[i] = geom_size[3 * g + i];
      o.cc[i] = -(C[i] * d[0] + C[3 + i] * d[1] + C[6 + i] * d[2]);
    }
    o.type = geom_type[g];
    o.dataid = o.type == MRS_GEOM_MESH ? mesh.dataid[g] : -1;
    for (int c = 0; c < 3; ++c) o.rgba[c] = geom_rgba[4 * g + c];
    const float s0 = o.size[0], s1 = o.size[1], s2 = o.size[2];
    float e[3] = {s0, s0, s0};
    switch (o.type) {
      case MRS_GEOM_BOX: case MRS_GEOM_ELLIPSOID: case MRS_GEOM_MESH: e[0] = s0; e[1] = s1; e[2] = s2; break;
      case MRS_GEOM_CAPSULE: e[2] = s1 + s0; break;
      case MRS_GEOM_CYLINDER: e[2] = s1; break;
      default: break;
    }
    for (int i = 0; i < 3; ++i) o.ext[i] = e[i] * 1.001f + 1e-4f;
    if (o.type == MRS_GEOM_PLANE && !(o.lp[2] > 0)) o.vis = 0;  // camera behind the plane
    if (o.type != MRS_GEOM_PLANE) {
      // view-axis extent of the oriented box: a geom wholly nearer than znear (e.g. the robot's own
      // body behind the camera) or wholly beyond zfar gives no pixel its depth -- hits nearer than
      // znear are discarded and hits beyond zfar read as zfar -- so it is dropped for the frame
      float rz = 0;
      for (int i = 0; i < 3; ++i) rz += o.ext[i] * fabsf(o.A[3 * i + 2]);
      const float zc = -o.cc[2];  // eye depth of the centre
      if (zc + rz < znear || zc - rz > zfar) o.vis = 0;
    }
  }
}
// shadow ray of the camera-frame kernels (lit_pixel's occluded): does a shadow-casting geom cross
// o + s L, 0 <= s < dist?  Geom-frame ray through the staged lp and A (a camera-frame point o maps to
// lp + A o); a bounding-sphere reject on the culling box first.  Oracle: ray_scene over groups 0-2.
template <bool kMesh = true>
__device__ inline bool occluded_staged(const DepthGeom* G, int ngeom, const MeshRef& mesh, const float o[3],
                                       const float L[3], float dist) {
  for (int k = 0; k < ngeom; ++k) {
    const DepthGeom& h = G[k];
    if (!h.cast) continue;
    if (h.type != MRS_GEOM_PLANE) {
      const float v[3] = {h.cc[0] - o[0], h.cc[1] - o[1], h.cc[2] - o[2]};
      const float r2 = h.ext[0] * h.ext[0] + h.ext[1] * h.ext[1] + h.ext[2] * h.ext[2];
      const float pr = v[0] * L[0] + v[1] * L[1] + v[2] * L[2];
      const float vv = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
      if (vv > r2 && (pr < 0 || vv - pr * pr > r2)) continue;  // origin outside, sphere behind or beside
    }
    float lp[3], lv[3];
    for (int i = 0; i < 3; ++i) {
      lp[i] = h.lp[i] + h.A[3 * i] * o[0] + h.A[3 * i + 1] * o[1] + h.A[3 * i + 2] * o[2];
      lv[i] = h.A[3 * i] * L[0] + h.A[3 * i + 1] * L[1] + h.A[3 * i + 2] * L[2];
    }
    float t;
    if (h.type == MRS_GEOM_BOX) t = ray_box_slab(h.size, lp, lv);
    else if (kMesh && h.type == MRS_GEOM_MESH) {
      int tri;
      t = ray_mesh(mesh.tri + 9 * mesh.faceadr[h.dataid], mesh.facenum[h.dataid], h.size, lp, lv,
                   mesh.bvh + 8 * mesh.bvhadr[h.dataid], mesh.bvhnum[h.dataid], &tri);
    } else t = ray_prim(h.type, h.size, lp, lv);
    if (t >= 0 && t < dist) return true;
  }
  return false;
}
#ifdef MRS_DEPTH_STATS
// diagnostics build: tiles, candidate visits and visits whose geom is the nearest hit of some pixel of
// the tile, summed over every frame (printed when the batch is freed)
__device__ unsigned long long g_depth_stats[4];
#endif
#ifndef MRS_DEPTH_MINBLK
#define MRS_DEPTH_MINBLK 1
#endif
// kMesh: the frame has mesh geoms (their per-pixel hierarchy walk, MRS_DEPTH_V2); frames without
// them take the instance without that code, whose registers allow more resident workgroups
template <bool kRGB, bool kMesh>
__global__ __launch_bounds__(256, MRS_DEPTH_MINBLK) void depth_kernel_v2(const int* geom_type, const int* geom_group,
                                                       const float* geom_size, const float* geom_rgba, int ngeom,
                                                       const float* geom_xpos, const float* geom_xmat,
                                                       const float* cam_xpos, const float* cam_xmat, int ncam, int cam,
                                                       int env0, int W, int H, float f, float znear, float zfar,
                                                       float* out, unsigned char* rgb, MeshRef mesh, LitRef lr) {
  __shared__ DepthGeom G[kDepthGeoms];
  __shared__ LitFrame LF;
  const int env = env0 + blockIdx.x;
  const size_t eo = static_cast<size_t>(env);
  const float* cp = cam_xpos + (eo * ncam + cam) * 3;
  const float* cm = cam_xmat + (eo * ncam + cam) * 9;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  stage_depth_geom(G, geom_type, geom_group, geom_size, geom_rgba, ngeom, geom_xpos, geom_xmat, cp, cm, eo, znear, zfar, mesh);
  if (kRGB && threadIdx.x == 64) lit_stage(LF, lr, cp, cm);
  __syncthreads();
  const int tiles_x = (W + kDepthTileW - 1) / kDepthTileW, tiles_y = (H + kDepthTileH - 1) / kDepthTileH;
  float* img = out + static_cast<size_t>(blockIdx.x) * W * H;
  for (int tile = wave; tile < tiles_x * tiles_y; tile += 4) {
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    // extreme pixel-centre ray slopes of the tile (camera frame: x right, y up, -z forward)
    const float x0 = (tx * kDepthTileW + 0.5f - 0.5f * W) / f;
    const float x1 = (fminf(tx * kDepthTileW + kDepthTileW - 1.0f, W - 1.0f) + 0.5f - 0.5f * W) / f;
    const float y1 = (0.5f * H - ty * kDepthTileH - 0.5f) / f;
    const float y0 = (0.5f * H - fminf(ty * kDepthTileH + kDepthTileH - 1.0f, H - 1.0f) - 0.5f) / f;
    bool keep = false;
    if (lane < ngeom && G[lane].vis) {
      const DepthGeom& o = G[lane];
      if (o.type == MRS_GEOM_PLANE) {
        // some corner ray (the minimum of the linear d.n over the tile) must descend onto the plane
        const float n[3] = {o.A[6], o.A[7], o.A[8]};
        const float bx = fminf(x0 * n[0], x1 * n[0]), by = fminf(y0 * n[1], y1 * n[1]);
        keep = bx + by - n[2] < 1e-6f;
      } else {
        // oriented box vs the four side planes n.p >= 0 of the tile pyramid (unnormalised normals:
        // left (1, 0, x0), right (-1, 0, -x1), bottom (0, 1, y0), top (0, -1, -y1))
        auto outside = [&](float nx, float ny, float nz) {
          const float c = nx * o.cc[0] + ny * o.cc[1] + nz * o.cc[2];
          float r = 0;
          for (int i = 0; i < 3; ++i)
            r += o.ext[i] * fabsf(nx * o.A[3 * i] + ny * o.A[3 * i + 1] + nz * o.A[3 * i + 2]);
          return c + r < -1e-5f * (fabsf(c) + r);
        };
        keep = !(outside(1, 0, x0) || outside(-1, 0, -x1) || outside(0, 1, y0) || outside(0, -1, -y1));
      }
    }
    unsigned long long cand = __ballot(keep);
    const int col = tx * kDepthTileW + lane;
    const float dx = (col + 0.5f - 0.5f * W) / f;
    const unsigned long long cand_tile = cand;
    // the tile's rows in chunks of kDepthChunk under the tile's one cull: only a chunk's rows are
    // live in registers (the fully unrolled 16-row tile held ~160 VGPRs, 3 workgroups per CU)
#pragma unroll 1
    for (int r0 = 0; r0 < kDepthTileH; r0 += kDepthChunk) {
    float best[kDepthChunk], dy[kDepthChunk];
    int bestg[kDepthChunk];
#pragma unroll
    for (int k = 0; k < kDepthChunk; ++k) {
      best[k] = -1;
      bestg[k] = 0;
      dy[k] = (0.5f * H - (ty * kDepthTileH + r0 + k) - 0.5f) / f;
    }
    cand = cand_tile;
    while (cand) {
      const int g = __builtin_ctzll(cand);
      cand &= cand - 1;
      const DepthGeom& o = G[g];
      const float lp[3] = {o.lp[0], o.lp[1], o.lp[2]}, sz[3] = {o.size[0], o.size[1], o.size[2]};
      float A[9];
      for (int i = 0; i < 9; ++i) A[i] = o.A[i];
      const int type = o.type;
#pragma unroll
      for (int k = 0; k < kDepthChunk; ++k) {
        float lv[3];
        pixel_ray(A, dx, dy[k], lv);
        float t;
        if (type == MRS_GEOM_BOX) t = ray_box_slab(sz, lp, lv);
        else if (kMesh && type == MRS_GEOM_MESH)
        {
          int tri;
          t = ray_mesh(mesh.tri + 9 * mesh.faceadr[o.dataid], mesh.facenum[o.dataid], sz, lp, lv,
                       mesh.bvh + 8 * mesh.bvhadr[o.dataid], mesh.bvhnum[o.dataid], &tri);
        }
        else t = ray_prim(type, sz, lp, lv);
        if (t >= znear && (best[k] < 0 || t < best[k])) { best[k] = t; bestg[k] = g; }
      }
    }
#ifdef MRS_DEPTH_STATS
    if (r0 == 0) {
      unsigned long long cc = cand_tile, won = 0;
      const int ncand = __popcll(cc);
      while (cc) {
        const int g = __builtin_ctzll(cc);
        cc &= cc - 1;
        bool w = false;
        for (int k = 0; k < kDepthChunk; ++k) w |= best[k] >= 0 && best[k] <= zfar && bestg[k] == g;
        if (__any(w)) ++won;
      }
      if (lane == 0) {
        atomicAdd(&g_depth_stats[0], 1ull);
        atomicAdd(&g_depth_stats[1], static_cast<unsigned long long>(ncand));
        atomicAdd(&g_depth_stats[2], won);
      }
    }
#endif
    if (col < W) {
#pragma unroll
      for (int k = 0; k < kDepthChunk; ++k) {
        const int row = ty * kDepthTileH + r0 + k;
        if (row < H) img[static_cast<size_t>(row) * W + col] = (best[k] < 0 || best[k] > zfar) ? zfar : best[k];
      }
      if constexpr (kRGB) {
        unsigned char* frame = rgb + static_cast<size_t>(blockIdx.x) * W * H * 3;
        for (int k = 0; k < kDepthChunk; ++k) {
          const int row = ty * kDepthTileH + r0 + k;
          if (row >= H) break;
          unsigned char* px = frame + (static_cast<size_t>(row) * W + col) * 3;
          if (best[k] < 0 || best[k] > zfar) { lit_sky(LF, dx, dy[k], px); continue; }
          const int g = bestg[k];
          const DepthGeom& o = G[g];
          // hit point in the geom frame lp + t lv; normal back to the camera frame through A's rows
          float q[3], nl[3], nc[3], lv[3];
          pixel_ray(o.A, dx, dy[k], lv);
          for (int i = 0; i < 3; ++i) q[i] = o.lp[i] + best[k] * lv[i];
          if (kMesh && o.type == MRS_GEOM_MESH) {  // the hit triangle's normal, facing the ray
            const float* mv = mesh.vert + 3 * mesh.vertadr[o.dataid];
            const int* mf = mesh.face + 3 * mesh.faceadr[o.dataid];
            int tri = 0;
            ray_mesh(mesh.tri + 9 * mesh.faceadr[o.dataid], mesh.facenum[o.dataid], o.size, o.lp, lv,
                     mesh.bvh + 8 * mesh.bvhadr[o.dataid], mesh.bvhnum[o.dataid], &tri);
            mesh_tri_normal(mv, mf, tri, lv, nl);
          } else {
            local_normal(o.type, o.size, q, nl);
          }
          for (int j = 0; j < 3; ++j) nc[j] = nl[0] * o.A[j] + nl[1] * o.A[3 + j] + nl[2] * o.A[6 + j];
          lit_pixel(LF, lr, g, o.rgba, o.type, o.size, q, dx, dy[k], best[k], nc,
                    [&](const float* so, const float* sl, float sd) { return occluded_staged<kMesh>(G, ngeom, mesh, so, sl, sd); },
                    px);
        }
      }
    }
    }
  }
}

// ---- frames of scenes with mesh geoms: triangle binning + per-pixel exact hits (depth_kernel_mesh).
// A per-pixel BVH walk (depth_kernel_v2's mesh path) is a chain of dependent node loads per pixel;
// here one workgroup renders one env frame in bands of kBandH rows:
//  1. every triangle of every visible mesh geom is put in camera coordinates once (lane per
//     triangle) and given its conservative pixel box (projected vertices, 1 pixel of margin);
//     triangles off screen, wholly nearer than znear or beyond zfar are dropped;
//  2. the kept triangles are sorted by first band (counting sort: per-band counters in LDS, the list
//     of (triangle, box) records in the frame's global scratch);
//  3. per band: each kept triangle overlapping the band tests the pixel rays of its box inside the
//     band with exactly raymesh.h ray_tri's arithmetic and keeps the nearest per pixel by an LDS
//     64-bit atomic min of (t bits, geom, triangle) -- so the depth of every pixel is bit-identical to
//     the every-triangle loop -- then every pixel of the band adds the primitive geoms (the band's
//     pyramid culls them as depth_kernel_v2's tile does), picks the nearest (ties to the lower geom
//     index, as the serial loop) and writes depth and colour.
// Triangles at or behind the camera plane, or spanning more than kMaxSpan bands, go to a side list
// tested in every band they overlap.
constexpr int kBandH = 8, kMaxBands = 128, kMaxSpan = 4;
constexpr int kRasterFaceBits = 18;  // triangle index bits in a record (mesh geom slot above)

// ray_tri (raymesh.h) with the triangle's vertex a and edges e1, e2 already loaded: the same
// expressions in the same order, so t is bit-identical
__device__ __forceinline__ float ray_tri_v(const float a[3], const float e1[3], const float e2[3], const float lp[3],
                                           const float lv[3]) {
  return mt_core(a, e1, e2, lp, lv);
}

struct TriLoad { float a[3], e1[3], e2[3]; };
__device__ __forceinline__ TriLoad load_tri(const float* rec, int f) {
  TriLoad o;
  for (int i = 0; i < 3; ++i) {
    o.a[i] = rec[9 * f + i];
    o.e1[i] = rec[9 * f + 3 + i];
    o.e2[i] = rec[9 * f + 6 + i];
  }
  return o;
}

// triangle f of mesh geom slot k: its conservative pixel box; 0 dropped, 1 kept, 2 side list
__device__ __forceinline__ int tri_box(const DepthGeom& o, const float* mv, const int* mf, int f, int W, int H, float fpx,
                                       float znear, float zfar, int& c0, int& c1, int& r0, int& r1) {
  const int id[3] = {3 * mf[3 * f], 3 * mf[3 * f + 1], 3 * mf[3 * f + 2]};
  float cmin = 3.0e38f, cmax = -3.0e38f, rmin = 3.0e38f, rmax = -3.0e38f, zmin = 3.0e38f, zmax = -3.0e38f;
  bool behind = false;
  for (int v = 0; v < 3; ++v) {
    const float q[3] = {mv[id[v]] - o.lp[0], mv[id[v] + 1] - o.lp[1], mv[id[v] + 2] - o.lp[2]};
    float c[3];
    for (int j = 0; j < 3; ++j) c[j] = o.A[j] * q[0] + o.A[3 + j] * q[1] + o.A[6 + j] * q[2];
    const float depth = -c[2];
    zmin = fminf(zmin, depth);
    zmax = fmaxf(zmax, depth);
    if (depth < 1e-4f) { behind = true; continue; }
    const float inv = fpx / depth;
    const float col = c[0] * inv + 0.5f * W - 0.5f, row = 0.5f * H - 0.5f - c[1] * inv;
    cmin = fminf(cmin, col); cmax = fmaxf(cmax, col);
    rmin = fminf(rmin, row); rmax = fmaxf(rmax, row);
  }
  // (1e-4 relative slack on the view-depth cull: t along the pixel ray equals the eye depth)
  if (zmax < znear * (1 - 1e-4f) || zmin > zfar * (1 + 1e-4f)) return 0;
  if (behind) { c0 = 0; c1 = W - 1; r0 = 0; r1 = H - 1; return 2; }
  c0 = max(0, static_cast<int>(ceilf(cmin)) - 1);
  c1 = min(W - 1, static_cast<int>(floorf(cmax)) + 1);
  r0 = max(0, static_cast<int>(ceilf(rmin)) - 1);
  r1 = min(H - 1, static_cast<int>(floorf(rmax)) + 1);
  if (c0 > c1 || r0 > r1) return 0;
  return (r1 / kBandH - r0 / kBandH) > kMaxSpan ? 2 : 1;
}

template <bool kRGB>
__global__ __launch_bounds__(256) void depth_kernel_mesh(const int* geom_type, const int* geom_group,
                                                         const float* geom_size, const float* geom_rgba, int ngeom,
                                                         const float* geom_xpos, const float* geom_xmat,
                                                         const float* cam_xpos, const float* cam_xmat, int ncam, int cam,
                                                         int env0, int W, int H, float f, float znear, float zfar,
                                                         float* out, unsigned char* rgb, MeshRef mesh, const int* mgeom,
                                                         const int* mbase, int nmg, int npair,
                                                         unsigned long long* lists, LitRef lr) {
  __shared__ DepthGeom G[kDepthGeoms];
  __shared__ LitFrame LF;
  __shared__ int cnt[kMaxBands + 1], cur[kMaxBands], mg[kDepthGeoms], mb[kDepthGeoms + 1];
  __shared__ int nside, maxspan;
  extern __shared__ unsigned long long band[];  // W x kBandH (t bits << 32 | geom << 24 | triangle)
  const int env = env0 + blockIdx.x;
  const size_t eo = static_cast<size_t>(env);
  const float* cp = cam_xpos + (eo * ncam + cam) * 3;
  const float* cm = cam_xmat + (eo * ncam + cam) * 9;
  const int lane = threadIdx.x & 63, tid = threadIdx.x;
  stage_depth_geom(G, geom_type, geom_group, geom_size, geom_rgba, ngeom, geom_xpos, geom_xmat, cp, cm, eo, znear, zfar, mesh);
  const int nb = (H + kBandH - 1) / kBandH;
  for (int i = tid; i <= nb; i += 256) cnt[i] = 0;
  for (int i = tid; i < nb; i += 256) cur[i] = 0;
  for (int i = tid; i < nmg; i += 256) { mg[i] = mgeom[i]; mb[i] = mbase[i]; }
  if (tid == 0) { mb[nmg] = npair; nside = 0; maxspan = 0; }
  if (kRGB && tid == 64) lit_stage(LF, lr, cp, cm);
  __syncthreads();
  unsigned long long* list = lists + static_cast<size_t>(blockIdx.x) * npair;
  // 1-2: count, then fill the band-sorted list (the side list fills the frame's list from its end)
  for (int pass = 0; pass < 2; ++pass) {
    int k = 0;
    for (int p = tid; p < npair; p += 256) {
      while (p >= mb[k + 1]) ++k;
      const DepthGeom& o = G[mg[k]];
      if (!o.vis) continue;
      const float* mv = mesh.vert + 3 * mesh.vertadr[o.dataid];
      const int* mf = mesh.face + 3 * mesh.faceadr[o.dataid];
      const int fi = p - mb[k];
      int c0, c1, r0, r1;
      const int kind = tri_box(o, mv, mf, fi, W, H, f, znear, zfar, c0, c1, r0, r1);
      if (kind == 0) continue;
      const int b0 = r0 / kBandH;
      if (pass == 0) {
        if (kind == 1) { atomicAdd(&cnt[b0], 1); atomicMax(&maxspan, r1 / kBandH - b0); }
        else atomicAdd(&nside, 1);
      } else {
        // record: triangle (24 bits: slot << kRasterFaceBits | index), c0 (11), c1 - c0 (11), r0 (10),
        // r1 - r0 (8; 255: to the last row, conservative for the side list)
        const unsigned long long rec = static_cast<unsigned long long>((k << kRasterFaceBits) | fi) |
                                       (static_cast<unsigned long long>(c0) << 24) |
                                       (static_cast<unsigned long long>(c1 - c0) << 35) |
                                       (static_cast<unsigned long long>(r0) << 46) |
                                       (static_cast<unsigned long long>(min(r1 - r0, 255)) << 56);
        if (kind == 1) list[cnt[b0] + atomicAdd(&cur[b0], 1)] = rec;
        else list[npair - 1 - atomicAdd(&nside, 1)] = rec;
      }
    }
    __syncthreads();
    if (pass == 0) {
      if (tid == 0) {  // exclusive prefix over the bands (cnt[b] becomes the band's first record)
        int acc = 0;
        for (int b = 0; b <= nb; ++b) { const int c = b < nb ? cnt[b] : 0; cnt[b] = acc; acc += c; }
        nside = 0;  // refilled by the fill pass
      }
      __syncthreads();
    }
  }
  __threadfence_block();
  __syncthreads();
  const int ms = maxspan, ns = nside;
  float* img = out + static_cast<size_t>(blockIdx.x) * W * H;
  unsigned char* frame = rgb ? rgb + static_cast<size_t>(blockIdx.x) * W * H * 3 : nullptr;
  const float x0 = (0.5f - 0.5f * W) / f, x1 = (W - 1.0f + 0.5f - 0.5f * W) / f;
  for (int b = 0; b < nb; ++b) {
    const int rb = b * kBandH, re = min(H, rb + kBandH);
    const int npx = (re - rb) * W;
    for (int i = tid; i < npx; i += 256) band[i] = ~0ull;
    __syncthreads();
    // 3a. triangles overlapping the band: band-sorted records of bands b - maxspan .. b, then the side list
    const int lo = cnt[max(0, b - ms)], hi = cnt[b + 1];
    const int nwork = hi - lo + ns;
    for (int w = tid; w < nwork; w += 256) {
      const unsigned long long rec = w < hi - lo ? list[lo + w] : list[npair - ns + (w - (hi - lo))];
      const int r0 = static_cast<int>((rec >> 46) & 0x3ff), dr = static_cast<int>(rec >> 56);
      const int r1 = dr == 255 ? H - 1 : r0 + dr;
      const int ra = max(r0, rb), rz = min(r1, re - 1);
      if (ra > rz) continue;
      const int c0 = static_cast<int>((rec >> 24) & 0x7ff), c1 = c0 + static_cast<int>((rec >> 35) & 0x7ff);
      const int kf = static_cast<int>(rec & 0xffffff), k = kf >> kRasterFaceBits, fi = kf & ((1 << kRasterFaceBits) - 1);
      const int g = mg[k];
      const DepthGeom& o = G[g];
      const TriLoad tr = load_tri(mesh.tri + 9 * mesh.faceadr[o.dataid], fi);
      const float lp[3] = {o.lp[0], o.lp[1], o.lp[2]};
      float A[9];
      for (int i = 0; i < 9; ++i) A[i] = o.A[i];
      const unsigned low = (static_cast<unsigned>(g) << 24) | static_cast<unsigned>(fi);
      for (int r = ra; r <= rz; ++r) {
        const float dy = (0.5f * H - r - 0.5f) / f;
        for (int c = c0; c <= c1; ++c) {
          const float dx = (c + 0.5f - 0.5f * W) / f;
          float lv[3];
        pixel_ray(A, dx, dy, lv);
          const float t = ray_tri_v(tr.a, tr.e1, tr.e2, lp, lv);
          if (t >= znear)
            atomicMin(&band[(r - rb) * W + c], (static_cast<unsigned long long>(__float_as_uint(t)) << 32) | low);
        }
      }
    }
    // 3b. primitive geoms of the band (pyramid cull as depth_kernel_v2's tile), then every pixel
    const float y1 = (0.5f * H - rb - 0.5f) / f, y0 = (0.5f * H - (re - 1) - 0.5f) / f;
    bool keep = false;
    if (lane < ngeom && G[lane].vis && G[lane].type != MRS_GEOM_MESH) {
      const DepthGeom& o = G[lane];
      if (o.type == MRS_GEOM_PLANE) {
        const float n[3] = {o.A[6], o.A[7], o.A[8]};
        const float bx = fminf(x0 * n[0], x1 * n[0]), by = fminf(y0 * n[1], y1 * n[1]);
        keep = bx + by - n[2] < 1e-6f;
      } else {
        auto outside = [&](float nx, float ny, float nz) {
          const float c = nx * o.cc[0] + ny * o.cc[1] + nz * o.cc[2];
          float r = 0;
          for (int i = 0; i < 3; ++i) r += o.ext[i] * fabsf(nx * o.A[3 * i] + ny * o.A[3 * i + 1] + nz * o.A[3 * i + 2]);
          return c + r < -1e-5f * (fabsf(c) + r);
        };
        keep = !(outside(1, 0, x0) || outside(-1, 0, -x1) || outside(0, 1, y0) || outside(0, -1, -y1));
      }
    }
    const unsigned long long prim = __ballot(keep);
    __syncthreads();
    for (int i = tid; i < npx; i += 256) {
      const int r = rb + i / W, c = i % W;
      const float dx = (c + 0.5f - 0.5f * W) / f, dy = (0.5f * H - r - 0.5f) / f;
      float best = -1;
      int bestg = 0;
      unsigned long long cand = prim;
      while (cand) {
        const int g = __builtin_ctzll(cand);
        cand &= cand - 1;
        const DepthGeom& o = G[g];
        const float lp[3] = {o.lp[0], o.lp[1], o.lp[2]}, sz[3] = {o.size[0], o.size[1], o.size[2]};
        float lv[3];
        pixel_ray(o.A, dx, dy, lv);
        const float t = o.type == MRS_GEOM_BOX ? ray_box_slab(sz, lp, lv) : ray_prim(o.type, sz, lp, lv);
        if (t >= znear && (best < 0 || t < best)) { best = t; bestg = g; }
      }
      const unsigned long long key = band[i];
      int tri = -1;
      if (key != ~0ull) {
        const float tm = __uint_as_float(static_cast<unsigned>(key >> 32));
        const int gm = static_cast<int>((key >> 24) & 0x3f);
        if (best < 0 || tm < best || (tm == best && gm < bestg)) {
          best = tm; bestg = gm; tri = static_cast<int>(key & 0xffffff);
        }
      }
      img[static_cast<size_t>(r) * W + c] = (best < 0 || best > zfar) ? zfar : best;
      if constexpr (kRGB) {
        unsigned char* px = frame + (static_cast<size_t>(r) * W + c) * 3;
        if (best < 0 || best > zfar) { lit_sky(LF, dx, dy, px); continue; }
        const DepthGeom& o = G[bestg];
        float lv[3], q[3];
        pixel_ray(o.A, dx, dy, lv);
        for (int k = 0; k < 3; ++k) q[k] = o.lp[k] + best * lv[k];
        float nl[3], nc[3];
        if (tri >= 0) {
          mesh_tri_normal(mesh.vert + 3 * mesh.vertadr[o.dataid], mesh.face + 3 * mesh.faceadr[o.dataid], tri, lv, nl);
        } else {
          local_normal(o.type, o.size, q, nl);
        }
        for (int j = 0; j < 3; ++j) nc[j] = nl[0] * o.A[j] + nl[1] * o.A[3 + j] + nl[2] * o.A[6 + j];
        lit_pixel(LF, lr, bestg, o.rgba, o.type, o.size, q, dx, dy, best, nc,
                  [&](const float* so, const float* sl, float sd) { return occluded_staged(G, ngeom, mesh, so, sl, sd); },
                  px);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ packing helpers
struct Packer {
  std::vector<float> f;
  std::vector<int> i;
  std::vector<std::pair<CPtr<float>*, size_t>> fptr;
  std::vector<std::pair<CPtr<int>*, size_t>> iptr;
  void addf(CPtr<float>* dst, const std::vector<double>& v) {
    fptr.emplace_back(dst, f.size());
    for (double x : v) f.push_back(static_cast<float>(x));
    while (f.size() % 4) f.push_back(0);
  }
  void addf(CPtr<float>* dst, const std::vector<float>& v) {
    fptr.emplace_back(dst, f.size());
    f.insert(f.end(), v.begin(), v.end());
    while (f.size() % 4) f.push_back(0);
  }
  void addi(CPtr<int>* dst, const std::vector<int>& v) {
    iptr.emplace_back(dst, i.size());
    i.insert(i.end(), v.begin(), v.end());
    while (i.size() % 4) i.push_back(0);
  }
};

}  // namespace

// ------------------------------------------------------------------ Batch implementation
struct BatchImpl {
  const Model* model = nullptr;
  int n = 0, device = 0;
  int group = 64;  // lanes per environment in the step kernel (64/group envs per wavefront)
  int g16_one_wg = 0;  // G = 16 with one workgroup per CU (tables past the two-per-CU budget)
  int wpb16 = WavesPerBlock<16>::value;  // waves per workgroup of the G = 16 kernels (DevState::wpb16)
  int helpers = 0;  // helper waves (DevState::ray_helpers), decided with the layout (build_devmodel)
  DevModel dm{};
  DevModel* d_dm = nullptr;  // device copy of dm
  LdsLayout& L = dm.L;
  ScratchLayout& S = dm.S;
  DevState st{};
  // a caller's device buffer [n][nu] the step launches read ctrl from (batch_bind_ctrl_device; null:
  // st.ctrl, the batch's own buffer)
  const float* ctrl_bound = nullptr;
  void* dblock_f = nullptr;
  void* dblock_i = nullptr;
  std::vector<void*> allocs;
  hipStream_t own_stream = nullptr, stream = nullptr;
  hipEvent_t ev0[2] = {nullptr, nullptr}, ev1[2] = {nullptr, nullptr};
  bool ev_valid[2] = {false, false};
  // launches bracketed by the batch's own HIP events for batch_last_kernel_ms: bit 0 step launches, bit 1
  // frames (batch_set_timing).  A timed step launch costs ~10 us (C3: 0.420 vs 0.410 ms per 10-step
  // launch), so step launches are timed only on request
  int timing = 2;
  std::vector<float> staging;
  std::vector<int> pair_g1, pair_g2;  // host copy of the static collision pairs (contact export)
  // camera pipeline (batch_render_async): pose snapshot + side stream, as the reference's rendering
  // thread renders its mjv_copyData snapshot while PhysicsLoop steps on (src/mujoco_cameras.cpp:204-215)
  hipStream_t rstream = nullptr;
  hipEvent_t snap_ev = nullptr, rend_ev = nullptr;
  bool rend_pending = false;
  float *snap_gpos = nullptr, *snap_gmat = nullptr, *snap_cpos = nullptr, *snap_cmat = nullptr;
  // depth_kernel_mesh: per-frame lists of (triangle, pixel box) records, sized for rast_frames frames
  unsigned long long* rast_list = nullptr;
  int rast_frames = 0;
  int max_lds = 0;  // hipDeviceAttributeMaxSharedMemoryPerBlock of the batch's device
  // the model needs the extended step kernels (step.hip MRS_EXT): general convex (MPR) collision
  // pairs, or rangefinders with more than 32 ray geoms
  bool ext = false;
};

namespace {

void* dalloc(BatchImpl& b, size_t bytes) {
  void* p = nullptr;
  HIP_CHECK(hipMalloc(&p, bytes ? bytes : 16));
  HIP_CHECK(hipMemsetAsync(p, 0, bytes ? bytes : 16, b.stream));
  b.allocs.push_back(p);
  return p;
}

// Per-mesh bounding volume hierarchy for rays (rangefinders, depth and colour): a binary tree over a
// mesh's triangles in depth-first order; each node stores its AABB, inflated by 1e-5 of the mesh's
// extent so that the fp32 slab test never rejects a triangle that Moller-Trumbore hits, and the index
// of the node after its subtree (stackless traversal, raymesh.h).  Leaves hold up to 4 consecutive
// triangles of the mesh's device face list, which is reordered for it (face ids stay relative to the
// mesh's vertices; only ties between triangles at equal ray parameter can pick a different triangle).
// Meshes of at most 64 triangles keep no hierarchy: a wave tests their triangles with scalar loads.
void build_mesh_bvh(const Model& m, std::vector<int>& face_out, std::vector<float>& node,
                    std::vector<int>& adr, std::vector<int>& num) {
  face_out = m.mesh_face;
  const int nmesh = static_cast<int>(m.mesh_faceadr.size());
  adr.assign(std::max(1, nmesh), 0);
  num.assign(std::max(1, nmesh), 0);
  auto fbits = [](int v) { float f; std::memcpy(&f, &v, sizeof f); return f; };
  for (int k = 0; k < nmesh; ++k) {
    const int fa = m.mesh_faceadr[k], fn = m.mesh_facenum[k], va = m.mesh_vertadr[k];
    adr[k] = static_cast<int>(node.size() / 8);
    if (fn <= 64 || std::getenv("MRS_NO_BVH")) continue;  // MRS_NO_BVH: every triangle (tests' A/B)
    struct Tri { double lo[3], hi[3], c[3]; int f[3]; };
    std::vector<Tri> tris(fn);
    double mlo[3] = {1e300, 1e300, 1e300}, mhi[3] = {-1e300, -1e300, -1e300};
    for (int f = 0; f < fn; ++f) {
      Tri& t = tris[f];
      for (int c = 0; c < 3; ++c) { t.lo[c] = 1e300; t.hi[c] = -1e300; t.f[c] = m.mesh_face[3 * (fa + f) + c]; }
      for (int v = 0; v < 3; ++v)
        for (int c = 0; c < 3; ++c) {
          const double x = m.mesh_vert[3 * (va + t.f[v]) + c];
          t.lo[c] = std::min(t.lo[c], x); t.hi[c] = std::max(t.hi[c], x);
        }
      for (int c = 0; c < 3; ++c) {
        t.c[c] = 0.5 * (t.lo[c] + t.hi[c]);
        mlo[c] = std::min(mlo[c], t.lo[c]); mhi[c] = std::max(mhi[c], t.hi[c]);
      }
    }
    const double pad = 1e-5 * std::max(1e-9, std::max(mhi[0] - mlo[0], std::max(mhi[1] - mlo[1], mhi[2] - mlo[2])));
    const int leaf = std::getenv("MRS_BVH_LEAF") ? std::max(1, std::min(64, std::atoi(std::getenv("MRS_BVH_LEAF")))) : 4;
    std::vector<float> nodes;
    std::function<void(int, int)> build = [&](int b, int e) {
      const int me = static_cast<int>(nodes.size() / 8);
      double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300}, clo[3] = {1e300, 1e300, 1e300},
             chi[3] = {-1e300, -1e300, -1e300};
      for (int i = b; i < e; ++i)
        for (int c = 0; c < 3; ++c) {
          lo[c] = std::min(lo[c], tris[i].lo[c]); hi[c] = std::max(hi[c], tris[i].hi[c]);
          clo[c] = std::min(clo[c], tris[i].c[c]); chi[c] = std::max(chi[c], tris[i].c[c]);
        }
      for (int c = 0; c < 3; ++c) nodes.push_back(static_cast<float>(lo[c] - pad));
      nodes.push_back(0);
      for (int c = 0; c < 3; ++c) nodes.push_back(static_cast<float>(hi[c] + pad));
      nodes.push_back(fbits(-1));
      if (e - b <= leaf) {
        nodes[8 * me + 7] = fbits((b << 8) | (e - b));
      } else {
        // binned surface-area heuristic (16 centroid bins per axis): the split minimising
        // N_left A_left + N_right A_right, i.e. the expected triangle tests of a ray that enters the
        // node; the median of the longest axis when no bin boundary separates the centroids
        constexpr int kBins = 16;
        auto area = [](const double* l, const double* h) {
          const double dx = h[0] - l[0], dy = h[1] - l[1], dz = h[2] - l[2];
          return dx * dy + dy * dz + dz * dx;
        };
        int best_ax = -1, best_s = 0;
        double best_cost = 1e300;
        for (int ax = 0; ax < 3; ++ax) {
          const double ext = chi[ax] - clo[ax];
          if (ext <= 1e-12) continue;
          int cnt[kBins] = {};
          double blo[kBins][3], bhi[kBins][3];
          for (int q = 0; q < kBins; ++q)
            for (int c = 0; c < 3; ++c) { blo[q][c] = 1e300; bhi[q][c] = -1e300; }
          for (int i = b; i < e; ++i) {
            const int q = std::min(kBins - 1, static_cast<int>((tris[i].c[ax] - clo[ax]) / ext * kBins));
            ++cnt[q];
            for (int c = 0; c < 3; ++c) { blo[q][c] = std::min(blo[q][c], tris[i].lo[c]); bhi[q][c] = std::max(bhi[q][c], tris[i].hi[c]); }
          }
          double rl[kBins][3], rh[kBins][3];
          int rn[kBins];
          for (int c = 0; c < 3; ++c) { rl[kBins - 1][c] = blo[kBins - 1][c]; rh[kBins - 1][c] = bhi[kBins - 1][c]; }
          rn[kBins - 1] = cnt[kBins - 1];
          for (int q = kBins - 2; q >= 0; --q) {
            rn[q] = rn[q + 1] + cnt[q];
            for (int c = 0; c < 3; ++c) { rl[q][c] = std::min(rl[q + 1][c], blo[q][c]); rh[q][c] = std::max(rh[q + 1][c], bhi[q][c]); }
          }
          double ll[3] = {1e300, 1e300, 1e300}, lh[3] = {-1e300, -1e300, -1e300};
          int ln = 0;
          for (int q = 1; q < kBins; ++q) {
            ln += cnt[q - 1];
            for (int c = 0; c < 3; ++c) { ll[c] = std::min(ll[c], blo[q - 1][c]); lh[c] = std::max(lh[c], bhi[q - 1][c]); }
            if (ln == 0 || rn[q] == 0) continue;
            const double cost = ln * area(ll, lh) + rn[q] * area(rl[q], rh[q]);
            if (cost < best_cost) { best_cost = cost; best_ax = ax; best_s = q; }
          }
        }
        int mid = (b + e) / 2;
        if (best_ax >= 0 && !std::getenv("MRS_BVH_MEDIAN")) {
          const double ext = chi[best_ax] - clo[best_ax];
          const int ax = best_ax, sp = best_s;
          const double lo0 = clo[ax];
          auto it = std::partition(tris.begin() + b, tris.begin() + e, [&](const Tri& t) {
            return std::min(kBins - 1, static_cast<int>((t.c[ax] - lo0) / ext * kBins)) < sp;
          });
          mid = static_cast<int>(it - tris.begin());
        } else {
          int ax = 0;
          for (int c = 1; c < 3; ++c)
            if (chi[c] - clo[c] > chi[ax] - clo[ax]) ax = c;
          std::nth_element(tris.begin() + b, tris.begin() + mid, tris.begin() + e,
                           [ax](const Tri& x, const Tri& y) { return x.c[ax] < y.c[ax]; });
        }
        build(b, mid);
        build(mid, e);
      }
      nodes[8 * me + 3] = fbits(static_cast<int>(nodes.size() / 8));
    };
    build(0, fn);
    for (int f = 0; f < fn; ++f)
      for (int c = 0; c < 3; ++c) face_out[3 * (fa + f) + c] = tris[f].f[c];
    num[k] = static_cast<int>(nodes.size() / 8);
    node.insert(node.end(), nodes.begin(), nodes.end());
  }
  if (node.empty()) node.assign(8, 0.0f);
}

void build_devmodel(BatchImpl& b, int max_con_req) {
  const Model& m = *b.model;
  DevModel& d = b.dm;
  if (m.nv > 64) throw UnsupportedError("nv > 64 is not supported by the one-wave-per-env kernel");
  for (int s = 0; s < m.nsensor; ++s) {
    int t = m.sensor_type[s];
    if (t == MRS_SENS_ACCELEROMETER) d.acc_sens |= 1;
    if (t == MRS_SENS_FORCE || t == MRS_SENS_TORQUE) d.acc_sens |= 3;
  }
  d.nq = m.nq; d.nv = m.nv; d.nu = m.nu; d.nbody = m.nbody; d.njnt = m.njnt; d.ngeom = m.ngeom;
  d.nsite = m.nsite; d.ncam = m.ncam; d.nsensor = m.nsensor; d.nsensordata = m.nsensordata;
  d.max_depth = m.max_depth;
  d.integrator = m.integrator; d.iterations = m.iterations; d.disableflags = m.disableflags;
  d.solver = m.solver; d.ls_iterations = m.ls_iterations; d.cone = m.cone; d.restate = m.restate;
  if (std::getenv("MRS_NO_MULTICCD")) d.restate |= MRS_RESTATE_NO_MULTICCD;  // (A/B of the face contacts)
  d.impratio = static_cast<float>(m.impratio); d.ls_tolerance = static_cast<float>(m.ls_tolerance);
  // diagnostic phase ablation for profiling only (bit 0 sensors, 1 collision, 2 constraints)
  d.diag_skip = std::getenv("MRS_DIAG_SKIP") ? std::atoi(std::getenv("MRS_DIAG_SKIP")) : 0;
  d.timestep = static_cast<float>(m.timestep);
  d.timestep_d = m.timestep;
  d.tolerance = static_cast<float>(m.tolerance);
  d.pgs_scale = static_cast<float>(1.0 / (m.stat_meaninertia * std::max(1, m.nv)));
  for (int i = 0; i < 3; ++i) d.gravity[i] = static_cast<float>(m.gravity[i]);

  // --- host precomputation of flat lists
  std::vector<int> subtree_end(m.nbody);
  for (int bI = m.nbody - 1; bI >= 0; --bI) {
    int e = bI + 1;
    while (e < m.nbody) {
      int x = e;
      bool inside = false;
      while (x != 0) { if (x == bI) { inside = true; break; } x = m.body_parentid[x]; }
      if (bI == 0) inside = true;
      if (!inside) break;
      ++e;
    }
    subtree_end[bI] = e;
  }
  std::vector<int> level_adr(m.max_depth + 2, 0), level_num(m.max_depth + 2, 0), level_body;
  for (int lev = 1; lev <= m.max_depth; ++lev) {
    level_adr[lev] = static_cast<int>(level_body.size());
    for (int bI = 1; bI < m.nbody; ++bI)
      if (m.body_depth[bI] == lev) level_body.push_back(bI);
    level_num[lev] = static_cast<int>(level_body.size()) - level_adr[lev];
  }
  // pointer-jumping tables for the tree passes: jump[r][b] = ancestor of b at distance 2^r when b
  // is deeper than 2^r (that ancestor is not the world body), else -1; ceil(log2(max_depth)) rounds
  d.kin_onepass = 1;
  for (int bI = 0; bI < m.nbody; ++bI) {
    const int nj = m.body_jntnum[bI];
    if (nj > 1) d.kin_onepass = 0;
    if (nj == 1) {
      const int t = m.jnt_type[m.body_jntadr[bI]];
      if (t != MRS_JNT_HINGE && t != MRS_JNT_FREE) d.kin_onepass = 0;
    }
  }
  if (std::getenv("MRS_KIN_TWOPASS")) d.kin_onepass = 0;  // A/B: the joint frames from a second pass
  d.njump = 0;
  while ((1 << d.njump) < m.max_depth) ++d.njump;
  std::vector<int> jump(std::max(1, d.njump * m.nbody), -1);
  for (int r = 0; r < d.njump; ++r)
    for (int bI = 1; bI < m.nbody; ++bI) {
      if (m.body_depth[bI] <= (1 << r)) continue;
      int a = bI;
      for (int k = 0; k < (1 << r); ++k) a = m.body_parentid[a];
      jump[r * m.nbody + bI] = a;
    }
  std::vector<int> Mpair;
  for (int i = 0; i < m.nv; ++i)
    for (int j = i; j >= 0; j = m.dof_parentid[j]) { Mpair.push_back(i); Mpair.push_back(j); }
  d.nMpair = static_cast<int>(Mpair.size() / 2);
  // static collision-pair filter (mj_collision broad phase minus the dynamic bounding test)
  std::vector<int> pg1, pg2, pdim;
  std::vector<float> pmargin, pgap, pfric, psolref, psolimp;
  {
    // explicit <contact><pair>s first, with their own parameters (mj_collision collides them before
    // the dynamic pairs; mrs::Model::expair_*)
    for (size_t q = 0; q < m.expair_geom1.size(); ++q) {
      const int ga = m.expair_geom1[q], gb = m.expair_geom2[q];
      const int ta = m.geom_type[ga], tb = m.geom_type[gb];
      if ((ta == MRS_GEOM_PLANE && tb == MRS_GEOM_PLANE) || ta == MRS_GEOM_HFIELD || tb == MRS_GEOM_HFIELD)
        throw UnsupportedError("explicit pair of geom types " + std::to_string(ta) + "/" + std::to_string(tb) +
                               " is not implemented");
      pg1.push_back(ga); pg2.push_back(gb);
      pdim.push_back(m.expair_dim[q]);
      pmargin.push_back(static_cast<float>(m.expair_margin[q]));
      pgap.push_back(static_cast<float>(m.expair_gap[q]));
      // (sliding, torsional, rolling) as the mixed pairs store them
      pfric.push_back(static_cast<float>(m.expair_friction[5 * q]));
      pfric.push_back(static_cast<float>(m.expair_friction[5 * q + 2]));
      pfric.push_back(static_cast<float>(m.expair_friction[5 * q + 3]));
      for (int i = 0; i < 2; ++i) psolref.push_back(static_cast<float>(m.expair_solref[2 * q + i]));
      for (int i = 0; i < 5; ++i) psolimp.push_back(static_cast<float>(m.expair_solimp[5 * q + i]));
    }
    // the compiler's statically admissible pairs (mrs::Model::pair_geom1/2, lower geom type first)
    for (size_t q = 0; q < m.pair_geom1.size(); ++q) {
        const int ga = m.pair_geom1[q], gb = m.pair_geom2[q];
        const int g1 = std::min(ga, gb), g2 = std::max(ga, gb);
        int ta = m.geom_type[ga], tb = m.geom_type[gb];
        // every pair of the implemented types: dedicated primitives, plane-ellipsoid/cylinder/mesh,
        // and MPR for the rest (step.hip narrowphase); plane-plane pairs (a plane on a moving body
        // against another plane) are skipped, as mj_collision has no plane-plane collider; hfields
        // are absent
        if (ta == MRS_GEOM_PLANE && tb == MRS_GEOM_PLANE) continue;
        bool ok = ta != MRS_GEOM_HFIELD && tb != MRS_GEOM_HFIELD;
        if (!ok)
          throw UnsupportedError("collision pair of geom types " + std::to_string(ta) + "/" + std::to_string(tb) +
                                 " is not implemented (geoms " + std::to_string(g1) + "," + std::to_string(g2) + ")");
        pg1.push_back(ga); pg2.push_back(gb);
        pdim.push_back(std::max(m.geom_condim[ga], m.geom_condim[gb]));
        pmargin.push_back(static_cast<float>(std::max(m.geom_margin[ga], m.geom_margin[gb])));
        pgap.push_back(static_cast<float>(std::max(m.geom_gap[ga], m.geom_gap[gb])));
        double s1 = m.geom_solmix[ga], s2 = m.geom_solmix[gb], mix;
        if (s1 >= 1e-15 && s2 >= 1e-15) mix = s1 / (s1 + s2);
        else if (s1 < 1e-15 && s2 < 1e-15) mix = 0.5;
        else mix = s1 < 1e-15 ? 0 : 1;
        for (int i = 0; i < 3; ++i)
          pfric.push_back(static_cast<float>(std::max(m.geom_friction[3 * ga + i], m.geom_friction[3 * gb + i])));
        for (int i = 0; i < 2; ++i)
          psolref.push_back(static_cast<float>(mix * m.geom_solref[2 * ga + i] + (1 - mix) * m.geom_solref[2 * gb + i]));
        for (int i = 0; i < 5; ++i)
          psolimp.push_back(static_cast<float>(mix * m.geom_solimp[5 * ga + i] + (1 - mix) * m.geom_solimp[5 * gb + i]));
      }
  }
  d.npair = static_cast<int>(pg1.size());
  b.pair_g1 = pg1;
  // active equality constraints (rows first in the solver order, as mj_makeConstraint)
  std::vector<int> eq_t, eq_o1, eq_o2;
  std::vector<double> eq_sr, eq_si, eq_dat;
  d.neq = d.neq_rows = 0;
  if (!(m.disableflags & (MRS_DSBL_EQUALITY | MRS_DSBL_CONSTRAINT)))
    for (size_t q = 0; q < m.eq_type.size(); ++q) {
      if (!m.eq_active0[q]) continue;
      eq_t.push_back(m.eq_type[q]); eq_o1.push_back(m.eq_obj1id[q]); eq_o2.push_back(m.eq_obj2id[q]);
      eq_sr.insert(eq_sr.end(), &m.eq_solref[2 * q], &m.eq_solref[2 * q] + 2);
      eq_si.insert(eq_si.end(), &m.eq_solimp[5 * q], &m.eq_solimp[5 * q] + 5);
      eq_dat.insert(eq_dat.end(), &m.eq_data[MRS_NEQDATA * q], &m.eq_data[MRS_NEQDATA * q] + MRS_NEQDATA);
      d.neq_rows += m.eq_type[q] == MRS_EQ_CONNECT ? 3 : (m.eq_type[q] == MRS_EQ_WELD ? 6 : 1);
    }
  d.neq = static_cast<int>(eq_t.size());
  // fixed tendons: wraps (qpos / dof address, coefficient), the constant Jacobian rows (dense
  // ntendon x nv), per tendon 12 constants (stiffness, damping, lengthspring[2], range[2], margin,
  // frictionloss, invweight0), and the tendons that give friction-loss / limit rows
  const int ntendon = static_cast<int>(m.tendon_adr.size());
  std::vector<int> ten_adr(m.tendon_adr), ten_num(m.tendon_num), wrap_qadr, wrap_dof, ten_fric, ten_lim;
  std::vector<double> wrap_coef(m.wrap_prm), tenJ(static_cast<size_t>(ntendon) * m.nv, 0.0), tenprm;
  for (size_t k = 0; k < m.wrap_objid.size(); ++k) {
    wrap_qadr.push_back(m.jnt_qposadr[m.wrap_objid[k]]);
    wrap_dof.push_back(m.jnt_dofadr[m.wrap_objid[k]]);
  }
  for (int t = 0; t < ntendon; ++t) {
    for (int k = m.tendon_adr[t]; k < m.tendon_adr[t] + m.tendon_num[t]; ++k)
      tenJ[static_cast<size_t>(t) * m.nv + wrap_dof[k]] += m.wrap_prm[k];
    const double pr[12] = {m.tendon_stiffness[t], m.tendon_damping[t], m.tendon_lengthspring[2 * t],
                           m.tendon_lengthspring[2 * t + 1], m.tendon_range[2 * t], m.tendon_range[2 * t + 1],
                           m.tendon_margin[t], m.tendon_frictionloss[t], m.tendon_invweight0[t], 0, 0, 0};
    tenprm.insert(tenprm.end(), pr, pr + 12);
    if (!(m.disableflags & (MRS_DSBL_FRICTIONLOSS | MRS_DSBL_CONSTRAINT)) && m.tendon_frictionloss[t] > 0)
      ten_fric.push_back(t);
    if (!(m.disableflags & (MRS_DSBL_LIMIT | MRS_DSBL_CONSTRAINT)) && m.tendon_limited[t]) ten_lim.push_back(t);
  }
  d.ntendon = ntendon;
  d.nten_fric = static_cast<int>(ten_fric.size());
  d.nten_lim = static_cast<int>(ten_lim.size());
  // rows outside the blocked-mode sparse solver's kinds (equality, tendon friction / limits): the
  // dense row path runs instead
  d.xrows = d.neq + d.nten_fric + d.nten_lim;
  b.pair_g2 = pg2;
  // kinematic trees (bodies sharing a root child of the world) that own dofs: their dofs are one
  // contiguous range, M is block diagonal over them, and constraint rows touch at most two of them
  // (mj_island's trees).  Blocked mode stores M / its factor per tree and solves the constraint rows
  // sparsely over the trees they touch (csrc/hip/step.hip constraints_sparse).
  std::vector<int> body_tree(m.nbody, -1), dof_tree(std::max(1, m.nv), -1), tree_dofadr, tree_dofnum, tree_Moff;
  {
    std::vector<int> root_tree(m.nbody, -1);
    for (int bI = 1; bI < m.nbody; ++bI) {
      if (m.body_dofnum[bI] == 0) continue;
      const int r = m.body_rootid[bI];
      if (root_tree[r] < 0) {
        root_tree[r] = static_cast<int>(tree_dofadr.size());
        tree_dofadr.push_back(m.body_dofadr[bI]);
        tree_dofnum.push_back(0);
      }
    }
    for (int bI = 1; bI < m.nbody; ++bI) body_tree[bI] = root_tree[m.body_rootid[bI]];
    for (int j = 0; j < m.nv; ++j) {
      const int t = body_tree[m.dof_bodyid[j]];
      if (t < 0 || j != tree_dofadr[t] + tree_dofnum[t])
        throw UnsupportedError("dofs of a kinematic tree are not contiguous");
      dof_tree[j] = t;
      ++tree_dofnum[t];
    }
    int off = 0;
    d.tree_nmax = 0;
    for (size_t t = 0; t < tree_dofadr.size(); ++t) {
      tree_Moff.push_back(off);
      off += tree_dofnum[t] * tree_dofnum[t];
      d.tree_nmax = std::max(d.tree_nmax, tree_dofnum[t]);
    }
    d.ntree = static_cast<int>(tree_dofadr.size());
    d.nMblk = off;
    // pipe width of the sparse solver: dof slots of the widest row (two trees for a contact)
    int widest = 1;
    for (int j = 0; j < m.nv; ++j) widest = std::max(widest, tree_dofnum[dof_tree[j]]);
    for (size_t p = 0; p < pg1.size(); ++p) {
      const int t1 = body_tree[m.geom_bodyid[pg1[p]]], t2 = body_tree[m.geom_bodyid[pg2[p]]];
      int w = (t1 >= 0 ? tree_dofnum[t1] : 0) + (t2 >= 0 && t2 != t1 ? tree_dofnum[t2] : 0);
      widest = std::max(widest, w);
    }
    d.pipe_w = 8;
    while (d.pipe_w < widest) d.pipe_w *= 2;
  }
  d.sparse_off = std::getenv("MRS_SPARSE_OFF") ? std::atoi(std::getenv("MRS_SPARSE_OFF")) & 15 : 0;
  std::vector<int> fric, lim, rf;
  for (int j = 0; j < m.nv; ++j) if (m.dof_frictionloss[j] > 0) fric.push_back(j);
  for (int j = 0; j < m.njnt; ++j)
    if (m.jnt_limited[j] && (m.jnt_type[j] == MRS_JNT_HINGE || m.jnt_type[j] == MRS_JNT_SLIDE)) lim.push_back(j);
  std::vector<int> other_sens;
  for (int s = 0; s < m.nsensor; ++s) {
    if (m.sensor_type[s] == MRS_SENS_RANGEFINDER) rf.push_back(s);
    else other_sens.push_back(s);
  }
  d.nsens_other = static_cast<int>(other_sens.size());
  d.nfric = static_cast<int>(fric.size());
  d.nlim = static_cast<int>(lim.size());
  d.nrf = static_cast<int>(rf.size());
  // contact capacity per env: requested, or (<= 0) the pairs' own maxima (8 for box-box and
  // plane-mesh, 4 for the other pairs) clamped to [32, 128]
  int pair_max = 0;
  for (size_t p = 0; p < pg1.size(); ++p) {
    const int ta = m.geom_type[pg1[p]], tb = m.geom_type[pg2[p]];
    pair_max += (ta == MRS_GEOM_BOX && tb == MRS_GEOM_BOX) || (ta == MRS_GEOM_PLANE && tb == MRS_GEOM_MESH) ? kMaxPairCon : 4;
  }
  const int cap = max_con_req > 0 ? max_con_req : std::min(128, std::max(32, pair_max));
  d.max_con = d.npair == 0 ? 0 : std::min(pair_max, cap);
  d.max_efc = d.neq_rows + d.nfric + d.nten_fric + 2 * (d.nlim + d.nten_lim) + 4 * d.max_con;
  // actuators
  std::vector<int> act_dof, act_qadr;
  std::vector<float> act_gear, act_gain, act_bias;
  std::vector<int> act_ten;
  for (int a = 0; a < m.nu; ++a) {
    int j = m.actuator_trnid[2 * a];
    if (m.actuator_trntype[a] == MRS_TRN_TENDON) {
      // a tendon transmission: the record's qpos / dof addresses hold -1 - tendon (length and
      // velocity from the step's tendon slot in LDS), its moment is gear * ten_J
      act_dof.push_back(-1 - j);
      act_qadr.push_back(-1 - j);
      act_ten.push_back(j);
    } else {
      if (m.jnt_type[j] != MRS_JNT_HINGE && m.jnt_type[j] != MRS_JNT_SLIDE)
        throw UnsupportedError("actuators on free/ball joints are not supported");
      act_dof.push_back(m.jnt_dofadr[j]);
      act_qadr.push_back(m.jnt_qposadr[j]);
      act_ten.push_back(-1);
    }
    act_gear.push_back(static_cast<float>(m.actuator_gear[6 * a]));
    for (int i = 0; i < 3; ++i) {
      act_gain.push_back(static_cast<float>(m.actuator_gainprm[MRS_NGAIN * a + i]));
      act_bias.push_back(static_cast<float>(m.actuator_biasprm[MRS_NBIAS * a + i]));
    }
  }

  Packer P;
  P.addi(&d.body_parentid, m.body_parentid); P.addi(&d.body_rootid, m.body_rootid);
  P.addi(&d.body_jntnum, m.body_jntnum); P.addi(&d.body_jntadr, m.body_jntadr);
  P.addi(&d.body_dofnum, m.body_dofnum); P.addi(&d.body_dofadr, m.body_dofadr);
  P.addi(&d.body_subtree_end, subtree_end); P.addi(&d.level_adr, level_adr);
  P.addi(&d.level_num, level_num); P.addi(&d.level_body, level_body); P.addi(&d.jump, jump);
  P.addf(&d.body_pos, m.body_pos); P.addf(&d.body_quat, m.body_quat); P.addf(&d.body_ipos, m.body_ipos);
  P.addf(&d.body_iquat, m.body_iquat); P.addf(&d.body_mass, m.body_mass);
  P.addf(&d.body_subtreemass, m.body_subtreemass); P.addf(&d.body_inertia, m.body_inertia);
  P.addf(&d.body_gravcomp, m.body_gravcomp); P.addf(&d.body_invweight0, m.body_invweight0);
  P.addi(&d.jnt_type, m.jnt_type); P.addi(&d.jnt_qposadr, m.jnt_qposadr); P.addi(&d.jnt_dofadr, m.jnt_dofadr);
  P.addi(&d.jnt_bodyid, m.jnt_bodyid); P.addi(&d.jnt_actfrclimited, m.jnt_actfrclimited);
  P.addf(&d.jnt_pos, m.jnt_pos); P.addf(&d.jnt_axis, m.jnt_axis); P.addf(&d.jnt_stiffness, m.jnt_stiffness);
  P.addf(&d.jnt_range, m.jnt_range); P.addf(&d.jnt_margin, m.jnt_margin); P.addf(&d.jnt_solref, m.jnt_solref);
  P.addf(&d.jnt_solimp, m.jnt_solimp); P.addf(&d.jnt_actfrcrange, m.jnt_actfrcrange);
  P.addi(&d.dof_bodyid, m.dof_bodyid); P.addi(&d.dof_jntid, m.dof_jntid);
  P.addf(&d.dof_armature, m.dof_armature); P.addf(&d.dof_damping, m.dof_damping);
  P.addf(&d.dof_frictionloss, m.dof_frictionloss); P.addf(&d.dof_solref, m.dof_solref);
  P.addf(&d.dof_solimp, m.dof_solimp); P.addf(&d.dof_invweight0, m.dof_invweight0);
  P.addf(&d.qpos0, m.qpos0); P.addf(&d.qpos_spring, m.qpos_spring);
  P.addi(&d.Mpair, Mpair);
  P.addi(&d.body_tree, body_tree); P.addi(&d.dof_tree, dof_tree); P.addi(&d.tree_dofadr, tree_dofadr);
  P.addi(&d.tree_dofnum, tree_dofnum); P.addi(&d.tree_Moff, tree_Moff);
  P.addi(&d.geom_type, m.geom_type); P.addi(&d.geom_bodyid, m.geom_bodyid); P.addi(&d.geom_group, m.geom_group);
  P.addi(&d.geom_dataid, m.geom_dataid);
  std::vector<int> bvh_face, bvh_adr, bvh_num;
  std::vector<float> bvh_node;
  build_mesh_bvh(m, bvh_face, bvh_node, bvh_adr, bvh_num);
  P.addi(&d.mesh_vertadr, m.mesh_vertadr); P.addi(&d.mesh_faceadr, m.mesh_faceadr); P.addi(&d.mesh_facenum, m.mesh_facenum);
  P.addi(&d.mesh_hulladr, m.mesh_hulladr); P.addi(&d.mesh_hullnum, m.mesh_hullnum); P.addi(&d.mesh_face, bvh_face);
  P.addi(&d.mesh_bvhadr, bvh_adr); P.addi(&d.mesh_bvhnum, bvh_num); P.addf(&d.mesh_bvh, bvh_node);
  P.addi(&d.mesh_hull, m.mesh_hull); P.addf(&d.mesh_vert, m.mesh_vert);
  P.addi(&d.mesh_polyadr, m.mesh_polyadr); P.addi(&d.mesh_polynum, m.mesh_polynum);
  P.addi(&d.mesh_polyvertadr, m.mesh_polyvertadr); P.addi(&d.mesh_polyvertnum, m.mesh_polynum_v);
  P.addi(&d.mesh_polyvert, m.mesh_polyvert); P.addf(&d.mesh_polynormal, m.mesh_polynormal);
  {
    // pre-gathered triangle records in device face order: vertex a, b - a, c - a, formed in fp32 from
    // the fp32 vertices exactly as ray_tri forms them on the device (bit-identical t)
    std::vector<float> tri(9 * bvh_face.size() / 3);
    const int nmesh = static_cast<int>(m.mesh_faceadr.size());
    for (int k = 0; k < nmesh; ++k)
      for (int f = m.mesh_faceadr[k]; f < m.mesh_faceadr[k] + m.mesh_facenum[k]; ++f) {
        float v[3][3];
        for (int c = 0; c < 3; ++c)
          for (int i = 0; i < 3; ++i) v[c][i] = static_cast<float>(m.mesh_vert[3 * (m.mesh_vertadr[k] + bvh_face[3 * f + c]) + i]);
        for (int i = 0; i < 3; ++i) {
          tri[9 * f + i] = v[0][i];
          tri[9 * f + 3 + i] = v[1][i] - v[0][i];
          tri[9 * f + 6 + i] = v[2][i] - v[0][i];
        }
      }
    P.addf(&d.mesh_tri, tri);
  }
  {
    // mesh geoms a camera can see (groups 0-2, alpha > 0), for the binning frame kernel; limits of its
    // records: 64 geom slots, 2^18 triangles per mesh, pairs within an int
    std::vector<int> rg, rb;
    long long np = 0;
    bool ok = true;
    for (int g = 0; g < m.ngeom; ++g) {
      if (m.geom_type[g] != MRS_GEOM_MESH || m.geom_group[g] < 0 || m.geom_group[g] > 2 || m.geom_rgba[4 * g + 3] == 0) continue;
      const int fn = m.mesh_facenum[m.geom_dataid[g]];
      ok &= fn < (1 << 18);
      rg.push_back(g);
      rb.push_back(static_cast<int>(np));
      np += fn;
    }
    ok &= rg.size() <= 64 && np < (1ll << 30) && m.ngeom <= kDepthGeoms;
    if (!ok) { rg.clear(); rb.clear(); np = 0; }
    d.nrast = static_cast<int>(rg.size());
    d.nrast_pair = static_cast<int>(np);
    P.addi(&d.rast_geom, rg); P.addi(&d.rast_base, rb);
  }
  P.addf(&d.geom_size, m.geom_size); P.addf(&d.geom_pos, m.geom_pos); P.addf(&d.geom_quat, m.geom_quat);
  P.addf(&d.geom_rbound, m.geom_rbound); P.addf(&d.geom_rgba, m.geom_rgba);
  {
    // lit.h's rlit block (layout in its header comment); more than kLitMaxLights lights are refused
    if (static_cast<int>(m.light_active.size()) > kLitMaxLights)
      throw std::runtime_error("at most " + std::to_string(kLitMaxLights) + " lights are supported");
    const int nl = static_cast<int>(m.light_active.size()), nm = static_cast<int>(m.mat_texid.size()),
              nt = static_cast<int>(m.tex_type.size());
    std::vector<double> r(kLitHead + kLitLight * nl + kLitMat * nm + kLitTex * nt, 0.0);
    for (int i = 0; i < 10; ++i) r[i] = m.vis_headlight[i];
    r[10] = nl;
    d.lit_sky = -1;
    for (int t = 0; t < nt && d.lit_sky < 0; ++t)
      if (m.tex_type[t] == MRS_TEX_SKYBOX) d.lit_sky = t;
    r[11] = d.lit_sky;
    for (int l = 0; l < nl; ++l) {
      double* o = r.data() + kLitHead + kLitLight * l;
      for (int i = 0; i < 3; ++i) {
        o[i] = m.light_pos[3 * l + i]; o[3 + i] = m.light_dir[3 * l + i];
        o[6 + i] = m.light_ambient[3 * l + i]; o[9 + i] = m.light_diffuse[3 * l + i];
        o[12 + i] = m.light_specular[3 * l + i]; o[15 + i] = m.light_attenuation[3 * l + i];
      }
      o[18] = std::cos(m.light_cutoff[l] * M_PI / 180); o[19] = m.light_exponent[l];
      o[20] = m.light_directional[l]; o[21] = m.light_castshadow[l]; o[22] = m.light_active[l];
    }
    d.lit_nlight = nl;
    d.lit_mat0 = kLitHead + kLitLight * nl;
    d.lit_tex0 = d.lit_mat0 + kLitMat * nm;
    for (int k = 0; k < nm; ++k) {
      double* o = r.data() + d.lit_mat0 + kLitMat * k;
      o[0] = m.mat_texid[k]; o[1] = m.mat_texuniform[k];
      o[2] = m.mat_texrepeat[2 * k]; o[3] = m.mat_texrepeat[2 * k + 1];
      o[4] = m.mat_specular[k]; o[5] = m.mat_shininess[k]; o[6] = m.mat_emission[k];
    }
    for (int t = 0; t < nt; ++t) {
      double* o = r.data() + d.lit_tex0 + kLitTex * t;
      o[0] = m.tex_type[t]; o[1] = m.tex_builtin[t]; o[2] = m.tex_mark[t];
      o[3] = m.tex_width[t]; o[4] = m.tex_height[t];
      for (int i = 0; i < 3; ++i) { o[5 + i] = m.tex_rgb1[3 * t + i]; o[8 + i] = m.tex_rgb2[3 * t + i]; o[11 + i] = m.tex_markrgb[3 * t + i]; }
    }
    P.addf(&d.rlit, r);
    std::vector<int> mid(m.ngeom, -1);
    for (int g = 0; g < m.ngeom && g < static_cast<int>(m.geom_matid.size()); ++g) mid[g] = m.geom_matid[g];
    P.addi(&d.geom_matid, mid);
  }
  P.addi(&d.pair_g1, pg1); P.addi(&d.pair_g2, pg2); P.addi(&d.pair_dim, pdim);
  P.addi(&d.ten_adr, ten_adr); P.addi(&d.ten_num, ten_num); P.addi(&d.wrap_qadr, wrap_qadr);
  P.addi(&d.wrap_dof, wrap_dof); P.addf(&d.wrap_coef, wrap_coef); P.addf(&d.ten_J, tenJ);
  P.addf(&d.ten_prm, tenprm); P.addi(&d.ten_fric, ten_fric); P.addi(&d.ten_lim, ten_lim);
  P.addf(&d.ten_solref_lim, m.tendon_solref_lim); P.addf(&d.ten_solimp_lim, m.tendon_solimp_lim);
  P.addf(&d.ten_solref_fri, m.tendon_solref_fri); P.addf(&d.ten_solimp_fri, m.tendon_solimp_fri);
  P.addi(&d.act_ten, act_ten);
  P.addi(&d.eq_type, eq_t); P.addi(&d.eq_obj1id, eq_o1); P.addi(&d.eq_obj2id, eq_o2);
  P.addf(&d.eq_solref, eq_sr); P.addf(&d.eq_solimp, eq_si); P.addf(&d.eq_data, eq_dat);
  P.addf(&d.pair_margin, pmargin); P.addf(&d.pair_gap, pgap); P.addf(&d.pair_friction, pfric);
  P.addf(&d.pair_solref, psolref); P.addf(&d.pair_solimp, psolimp);
  P.addi(&d.site_bodyid, m.site_bodyid); P.addf(&d.site_pos, m.site_pos); P.addf(&d.site_quat, m.site_quat);
  P.addi(&d.cam_bodyid, m.cam_bodyid); P.addf(&d.cam_pos, m.cam_pos); P.addf(&d.cam_quat, m.cam_quat);
  P.addi(&d.act_dof, act_dof); P.addi(&d.act_qadr, act_qadr);
  P.addi(&d.act_gaintype, m.actuator_gaintype); P.addi(&d.act_biastype, m.actuator_biastype);
  P.addi(&d.act_ctrllimited, m.actuator_ctrllimited); P.addi(&d.act_forcelimited, m.actuator_forcelimited);
  P.addf(&d.act_gear, act_gear); P.addf(&d.act_gainprm, act_gain); P.addf(&d.act_biasprm, act_bias);
  P.addf(&d.act_ctrlrange, m.actuator_ctrlrange); P.addf(&d.act_forcerange, m.actuator_forcerange);
  P.addi(&d.sensor_type, m.sensor_type); P.addi(&d.sensor_objtype, m.sensor_objtype);
  P.addi(&d.sensor_objid, m.sensor_objid); P.addi(&d.sensor_adr, m.sensor_adr); P.addi(&d.sensor_dim, m.sensor_dim);
  P.addf(&d.sensor_cutoff, m.sensor_cutoff);
  P.addi(&d.fric_dof, fric); P.addi(&d.lim_jnt, lim); P.addi(&d.rf_sensor, rf);
  P.addi(&d.sens_other, other_sens);
  // friction-loss rows and limited joints, 4 floats each, staged in workgroup LDS (shr_fric, shr_lim):
  // a friction row's impedance is that of distance 0 at margin 0, so its R and reference stiffness
  // B are model constants (computed here in fp32, the order the kernel used); limits: qpos address,
  // margin, range
  std::vector<float> fricrec, limrec;
  {
    auto fbits = [](int v) { float f; std::memcpy(&f, &v, sizeof f); return f; };
    auto clampf = [](float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); };
    for (int j : fric) {
      const float si0 = static_cast<float>(m.dof_solimp[5 * j]), si1 = static_cast<float>(m.dof_solimp[5 * j + 1]);
      const float width = static_cast<float>(m.dof_solimp[5 * j + 2]);
      const float dmin = clampf(si0, 0.0001f, 0.9999f), dmax = clampf(si1, 0.0001f, 0.9999f);
      const float imp = (dmin == dmax || width <= 1e-15f) ? 0.5f * (dmin + dmax) : dmin;
      float R = (1 - imp) * static_cast<float>(m.dof_invweight0[j]) / imp;
      R = R > 1e-15f ? R : 1e-15f;
      const float sr0 = static_cast<float>(m.dof_solref[2 * j]), sr1 = static_cast<float>(m.dof_solref[2 * j + 1]);
      float B;
      if (sr0 > 0) {
        float tc = sr0;
        if (!(m.disableflags & MRS_DSBL_REFSAFE) && tc < 2 * d.timestep) tc = 2 * d.timestep;
        B = 2 / (dmax * tc);
      } else {
        B = -sr1 / dmax;
      }
      fricrec.insert(fricrec.end(), {fbits(j), R, B, static_cast<float>(m.dof_frictionloss[j])});
    }
    for (int j : lim)
      limrec.insert(limrec.end(), {fbits(m.jnt_qposadr[j]), static_cast<float>(m.jnt_margin[j]),
                                   static_cast<float>(m.jnt_range[2 * j]), static_cast<float>(m.jnt_range[2 * j + 1])});
  }
  P.addf(&d.fricrec, fricrec);
  P.addf(&d.limrec, limrec);
  // smooth-force tables (step.hip smooth_forces), staged in workgroup LDS: per actuator (20 floats)
  // qpos / dof address, gear, ctrl limit flag and range, gain type and prm[3], bias type and prm[3],
  // force limit flag and range; per dof (16 floats) its single actuator (-1 none, -2 several: the
  // actuator loop runs), that actuator's gear, the joint's actuator-force limit flag and range,
  // joint type, stiffness, qpos address, qpos_spring, the dof's damping, body, subtree end,
  // whether any body of the subtree has gravcomp, the dof's friction-loss row (-1 none) and its
  // joint's first dof
  std::vector<float> actrec, dofrec;
  {
    auto fbits = [](int v) { float f; std::memcpy(&f, &v, sizeof f); return f; };
    for (int a = 0; a < m.nu; ++a) {
      std::vector<float> r = {fbits(act_qadr[a]), fbits(act_dof[a]), act_gear[a], fbits(m.actuator_ctrllimited[a]),
                              static_cast<float>(m.actuator_ctrlrange[2 * a]), static_cast<float>(m.actuator_ctrlrange[2 * a + 1]),
                              fbits(m.actuator_gaintype[a]), act_gain[3 * a], act_gain[3 * a + 1], act_gain[3 * a + 2],
                              fbits(m.actuator_biastype[a]), act_bias[3 * a], act_bias[3 * a + 1], act_bias[3 * a + 2],
                              fbits(m.actuator_forcelimited[a]), static_cast<float>(m.actuator_forcerange[2 * a]),
                              static_cast<float>(m.actuator_forcerange[2 * a + 1]), 0.0f, 0.0f, 0.0f};
      actrec.insert(actrec.end(), r.begin(), r.end());
    }
    // each dof's friction-loss row (its index in the friction rows, -1 none): the 16-lane register
    // solvers index the friction rows by dof (step.hip constraints)
    std::vector<int> fric_row(m.nv, -1);
    for (size_t k = 0; k < fric.size(); ++k) fric_row[fric[k]] = static_cast<int>(k);
    for (int j = 0; j < m.nv; ++j) {
      int act = -1;
      float gear = 0;
      for (int a = 0; a < m.nu; ++a) {
        if (act_dof[a] == j) { act = act == -1 ? a : -2; gear = act_gear[a]; }
        if (act_ten[a] >= 0 && tenJ[static_cast<size_t>(act_ten[a]) * m.nv + j] != 0) act = -2;  // the loop
      }
      const int jid = m.dof_jntid[j], b = m.dof_bodyid[j];
      int gc = 0;
      for (int x = b; x < subtree_end[b]; ++x) gc |= m.body_gravcomp[x] != 0;
      std::vector<float> r = {fbits(act), gear, fbits(m.jnt_actfrclimited[jid]), static_cast<float>(m.jnt_actfrcrange[2 * jid]),
                              static_cast<float>(m.jnt_actfrcrange[2 * jid + 1]), fbits(m.jnt_type[jid]),
                              static_cast<float>(m.jnt_stiffness[jid]), fbits(m.jnt_qposadr[jid]),
                              static_cast<float>(m.qpos_spring[m.jnt_qposadr[jid]]), static_cast<float>(m.dof_damping[j]),
                              fbits(b), fbits(subtree_end[b]), fbits(gc), fbits(fric_row[j]),
                              fbits(m.jnt_dofadr[jid]), 0.0f};
      dofrec.insert(dofrec.end(), r.begin(), r.end());
    }
  }
  P.addf(&d.actrec, actrec);
  P.addf(&d.dofrec, dofrec);
  // tree tables for the smooth dynamics (step.hip com_pos, make_M, com_vel, rne), staged in workgroup
  // LDS: per body (8 floats) mass, subtree mass, root, parent, subtree end, dof address, dof count,
  // pad; per (dof, ancestor-dof) pair of M (4 floats) i, j, body of i, armature when i == j
  std::vector<float> bodytab, mpairtab;
  {
    auto fbits = [](int v) { float f; std::memcpy(&f, &v, sizeof f); return f; };
    for (int b = 0; b < m.nbody; ++b)
      bodytab.insert(bodytab.end(), {static_cast<float>(m.body_mass[b]), static_cast<float>(m.body_subtreemass[b]),
                                     fbits(m.body_rootid[b]), fbits(m.body_parentid[b]), fbits(subtree_end[b]),
                                     fbits(m.body_dofadr[b]), fbits(m.body_dofnum[b]), 0.0f});
    for (size_t q = 0; q + 1 < Mpair.size(); q += 2) {
      const int i = Mpair[q], j = Mpair[q + 1];
      mpairtab.insert(mpairtab.end(), {fbits(i), fbits(j), fbits(m.dof_bodyid[i]),
                                       i == j ? static_cast<float>(m.dof_armature[i]) : 0.0f});
    }
  }
  P.addf(&d.bodytab, bodytab);
  P.addf(&d.mpairtab, mpairtab);
  // kinematics tables (step.hip body_pose / body_frame_out / kinematics / com_pos), staged in workgroup
  // LDS with lane groups: per body (25 floats) pos[3], quat[4], ipos[3], iquat[4], inertia[3], first
  // joint, joint count (int bits), pad; per joint (13) pos[3], axis[3], qpos address, type, qpos0 of
  // the address, body, dof address, the body's root (int bits), pad; per geom (9) body (int bits),
  // pos[3], quat[4], pad
  {
    auto fbits = [](int v) { float f; std::memcpy(&f, &v, sizeof f); return f; };
    std::vector<float> kb, kj, kg;
    for (int b = 0; b < m.nbody; ++b) {
      for (int i = 0; i < 3; ++i) kb.push_back(static_cast<float>(m.body_pos[3 * b + i]));
      for (int i = 0; i < 4; ++i) kb.push_back(static_cast<float>(m.body_quat[4 * b + i]));
      for (int i = 0; i < 3; ++i) kb.push_back(static_cast<float>(m.body_ipos[3 * b + i]));
      for (int i = 0; i < 4; ++i) kb.push_back(static_cast<float>(m.body_iquat[4 * b + i]));
      for (int i = 0; i < 3; ++i) kb.push_back(static_cast<float>(m.body_inertia[3 * b + i]));
      kb.push_back(fbits(m.body_jntadr[b]));
      kb.push_back(fbits(m.body_jntnum[b]));
      while (kb.size() % 25) kb.push_back(0.0f);
    }
    for (int j = 0; j < m.njnt; ++j) {
      for (int i = 0; i < 3; ++i) kj.push_back(static_cast<float>(m.jnt_pos[3 * j + i]));
      for (int i = 0; i < 3; ++i) kj.push_back(static_cast<float>(m.jnt_axis[3 * j + i]));
      kj.push_back(fbits(m.jnt_qposadr[j]));
      kj.push_back(fbits(m.jnt_type[j]));
      kj.push_back(static_cast<float>(m.qpos0[m.jnt_qposadr[j]]));
      kj.push_back(fbits(m.jnt_bodyid[j]));
      kj.push_back(fbits(m.jnt_dofadr[j]));
      kj.push_back(fbits(m.body_rootid[m.jnt_bodyid[j]]));
      while (kj.size() % 13) kj.push_back(0.0f);
    }
    for (int g = 0; g < m.ngeom; ++g) {
      kg.push_back(fbits(m.geom_bodyid[g]));
      for (int i = 0; i < 3; ++i) kg.push_back(static_cast<float>(m.geom_pos[3 * g + i]));
      for (int i = 0; i < 4; ++i) kg.push_back(static_cast<float>(m.geom_quat[4 * g + i]));
      kg.push_back(0.0f);
    }
    P.addf(&d.kinbody, kb);
    P.addf(&d.kinjnt, kj);
    P.addf(&d.kingeom, kg);
  }
  // the non-ray sensors' descriptors, 16 floats each (staged in workgroup LDS at shr_sens): type,
  // objtype, sensordata address, dim (int bits), cutoff, the object's qpos / dof / actuator / body
  // index (int bits), the root body (int bits), then the site's or geom's local pos[3] and quat[4]
  std::vector<float> sensrec;
  {
    auto fbits = [](int v) { float f; std::memcpy(&f, &v, sizeof f); return f; };
    for (int sid : other_sens) {
      const int t = m.sensor_type[sid], ot = m.sensor_objtype[sid], id = m.sensor_objid[sid];
      int a = id, root = 0;
      double lp[3] = {0, 0, 0}, lq[4] = {1, 0, 0, 0};
      if (t == MRS_SENS_JOINTPOS) a = m.jnt_qposadr[id];
      else if (t == MRS_SENS_JOINTVEL) a = m.jnt_dofadr[id];
      else if (t == MRS_SENS_ACCELEROMETER || t == MRS_SENS_FORCE || t == MRS_SENS_TORQUE || t == MRS_SENS_GYRO ||
               ((t == MRS_SENS_FRAMEPOS || t == MRS_SENS_FRAMEQUAT) && ot == MRS_OBJ_SITE)) {
        a = m.site_bodyid[id];
        for (int i = 0; i < 3; ++i) lp[i] = m.site_pos[3 * id + i];
        for (int i = 0; i < 4; ++i) lq[i] = m.site_quat[4 * id + i];
      } else if ((t == MRS_SENS_FRAMEPOS || t == MRS_SENS_FRAMEQUAT) && ot != MRS_OBJ_BODY) {  // geom
        a = m.geom_bodyid[id];
        for (int i = 0; i < 4; ++i) lq[i] = m.geom_quat[4 * id + i];
      }
      if (a >= 0 && (t == MRS_SENS_ACCELEROMETER || t == MRS_SENS_FORCE || t == MRS_SENS_TORQUE)) root = m.body_rootid[a];
      sensrec.insert(sensrec.end(), {fbits(t), fbits(ot), fbits(m.sensor_adr[sid]), fbits(m.sensor_dim[sid]),
                                     static_cast<float>(m.sensor_cutoff[sid]), fbits(a), fbits(root),
                                     static_cast<float>(lp[0]), static_cast<float>(lp[1]), static_cast<float>(lp[2]),
                                     static_cast<float>(lq[0]), static_cast<float>(lq[1]), static_cast<float>(lq[2]),
                                     static_cast<float>(lq[3]), fbits(id), 0.0f});
    }
  }
  P.addf(&d.sensrec, sensrec);
  std::vector<float> rgeom;
  auto bits = [](int v) { float f; std::memcpy(&f, &v, sizeof f); return f; };
  for (int g = 0; g < m.ngeom; ++g) {
    if (m.geom_rgba[4 * g + 3] == 0) continue;
    rgeom.insert(rgeom.end(), {bits(g), bits(m.geom_type[g]), bits(m.geom_bodyid[g]),
                               static_cast<float>(m.geom_rbound[g]), static_cast<float>(m.geom_size[3 * g]),
                               static_cast<float>(m.geom_size[3 * g + 1]), static_cast<float>(m.geom_size[3 * g + 2]),
                               bits(m.geom_dataid[g])});
  }
  d.nrgeom = static_cast<int>(rgeom.size() / 8);
  P.addf(&d.rgeom, rgeom);
  // ray blocks (kRayBlock consecutive rangefinders) for the level-1 cull.  When every ray of a block
  // starts at the same point of the same body the block is bounded by a fan fixed in that body's
  // frame: unit axis a, in-plane direction b and normal c (the least-spread direction of the rays),
  // in-plane half-angle theta around a and out-of-plane slope eps = max |d.c| (a planar lidar fan
  // has eps ~ 0).  Blocks without a common origin, or wider than +-80 degrees, test every geom.
  std::vector<float> rfblk, rfblk_eps;
  d.nrfblk = 0;
  if (d.nrgeom <= 32 && d.nrf > 0) {
    d.nrfblk = (d.nrf + kRayBlock - 1) / kRayBlock;
    for (int blk = 0; blk < d.nrfblk; ++blk) {
      const int k0 = blk * kRayBlock, k1 = std::min(d.nrf, k0 + kRayBlock);
      const int site0 = m.sensor_objid[rf[k0]], body = m.site_bodyid[site0];
      bool ok = true;
      std::vector<std::array<double, 3>> dirs;
      double axis[3] = {0, 0, 0}, cov[3][3] = {};
      for (int k = k0; k < k1; ++k) {
        const int site = m.sensor_objid[rf[k]];
        if (m.site_bodyid[site] != body) ok = false;
        for (int i = 0; i < 3; ++i)
          if (std::abs(m.site_pos[3 * site + i] - m.site_pos[3 * site0 + i]) > 1e-9) ok = false;
        const double* q = &m.site_quat[4 * site];  // z column of the site rotation (ray direction)
        std::array<double, 3> dz = {2 * (q[1] * q[3] + q[0] * q[2]), 2 * (q[2] * q[3] - q[0] * q[1]),
                                    q[0] * q[0] - q[1] * q[1] - q[2] * q[2] + q[3] * q[3]};
        const double n = std::sqrt(dz[0] * dz[0] + dz[1] * dz[1] + dz[2] * dz[2]);
        for (int i = 0; i < 3; ++i) { dz[i] /= n; axis[i] += dz[i]; }
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) cov[i][j] += dz[i] * dz[j];
        dirs.push_back(dz);
      }
      double an = std::sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
      double c[3] = {0, 0, 1}, bv[3] = {0, 1, 0}, theta = 0, eps = 0;
      if (an < 1e-6) ok = false;
      if (ok) {
        for (int i = 0; i < 3; ++i) axis[i] /= an;
        // normal of the fan: eigenvector of the smallest eigenvalue of sum d d' (cyclic Jacobi)
        double A[3][3], V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        std::memcpy(A, cov, sizeof A);
        for (int sweep = 0; sweep < 50; ++sweep)
          for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
              if (std::abs(A[p][q]) < 1e-15) continue;
              const double th = 0.5 * std::atan2(2 * A[p][q], A[q][q] - A[p][p]);
              const double cs = std::cos(th), sn = std::sin(th);
              for (int k = 0; k < 3; ++k) {
                const double akp = A[k][p], akq = A[k][q];
                A[k][p] = cs * akp - sn * akq; A[k][q] = sn * akp + cs * akq;
              }
              for (int k = 0; k < 3; ++k) {
                const double apk = A[p][k], aqk = A[q][k];
                A[p][k] = cs * apk - sn * aqk; A[q][k] = sn * apk + cs * aqk;
              }
              for (int k = 0; k < 3; ++k) {
                const double vkp = V[k][p], vkq = V[k][q];
                V[k][p] = cs * vkp - sn * vkq; V[k][q] = sn * vkp + cs * vkq;
              }
            }
        int imin = 0;
        for (int i = 1; i < 3; ++i) if (A[i][i] < A[imin][imin]) imin = i;
        for (int i = 0; i < 3; ++i) c[i] = V[i][imin];
        const double ca = c[0] * axis[0] + c[1] * axis[1] + c[2] * axis[2];
        for (int i = 0; i < 3; ++i) c[i] -= ca * axis[i];
        const double cn = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
        if (cn < 1e-6) ok = false;
        else {
          for (int i = 0; i < 3; ++i) c[i] /= cn;
          bv[0] = c[1] * axis[2] - c[2] * axis[1];
          bv[1] = c[2] * axis[0] - c[0] * axis[2];
          bv[2] = c[0] * axis[1] - c[1] * axis[0];
          for (auto& dz : dirs) {
            const double da = dz[0] * axis[0] + dz[1] * axis[1] + dz[2] * axis[2];
            const double db = dz[0] * bv[0] + dz[1] * bv[1] + dz[2] * bv[2];
            const double dc = dz[0] * c[0] + dz[1] * c[1] + dz[2] * c[2];
            theta = std::max(theta, std::abs(std::atan2(db, da)));
            eps = std::max(eps, std::abs(dc));
          }
          if (theta > 1.4) ok = false;
        }
      }
      rfblk.insert(rfblk.end(), {bits(body), bits(ok ? 1 : 0), static_cast<float>(m.site_pos[3 * site0]),
                                 static_cast<float>(m.site_pos[3 * site0 + 1]), static_cast<float>(m.site_pos[3 * site0 + 2]),
                                 static_cast<float>(axis[0]), static_cast<float>(axis[1]), static_cast<float>(axis[2]),
                                 static_cast<float>(bv[0]), static_cast<float>(bv[1]), static_cast<float>(bv[2]),
                                 static_cast<float>(c[0]), static_cast<float>(c[1]), static_cast<float>(c[2]),
                                 static_cast<float>(std::cos(theta + 1e-4)), static_cast<float>(std::sin(theta + 1e-4))});
      rfblk_eps.push_back(static_cast<float>(eps + 1e-6));
    }
  }
  // record: body, flag, origin[3], a[3], b[3], c[3], cos(theta), sin(theta); then eps per block
  rfblk.insert(rfblk.end(), rfblk_eps.begin(), rfblk_eps.end());
  // every ray of the lidar(s) from one point of one body: the pass loop reuses one frame
  d.rf_common = d.nrfblk > 0 ? 1 : 0;
  for (int blk = 0; blk < d.nrfblk && d.rf_common; ++blk) {
    const float* r0 = &rfblk[0];
    const float* ri = &rfblk[16 * blk];
    int f; std::memcpy(&f, &ri[1], 4);
    if (!f || std::memcmp(&ri[0], &r0[0], 4) != 0 || ri[2] != r0[2] || ri[3] != r0[3] || ri[4] != r0[4]) d.rf_common = 0;
  }
  // static lidars: when every rangefinder sits on a world-welded body, that body's world pose never
  // changes, so the ray blocks' fan frames and the rays' origins / directions go to the world frame
  // here (fp64) and the step kernel skips the per-step body rotation (rf_static_frame)
  d.rf_static_frame = 0;
  if (d.nrf > 0) {
    bool all_static = true;
    for (int k = 0; k < d.nrf; ++k) all_static = all_static && m.body_weldid[m.site_bodyid[m.sensor_objid[rf[k]]]] == 0;
    d.rf_static_frame = all_static && !std::getenv("MRS_NO_STATIC_FRAME") ? 1 : 0;
  }
  auto body_world = [&](int b, double R[9], double p[3]) {  // world pose of a body without joints above it
    double q[4] = {1, 0, 0, 0};
    p[0] = p[1] = p[2] = 0;
    std::vector<int> chain;
    for (int x = b; x != 0; x = m.body_parentid[x]) chain.push_back(x);
    for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
      const double* bp = &m.body_pos[3 * *it];
      const double* bq = &m.body_quat[4 * *it];
      const double Rq[9] = {q[0] * q[0] + q[1] * q[1] - q[2] * q[2] - q[3] * q[3], 2 * (q[1] * q[2] - q[0] * q[3]),
                            2 * (q[1] * q[3] + q[0] * q[2]), 2 * (q[1] * q[2] + q[0] * q[3]),
                            q[0] * q[0] - q[1] * q[1] + q[2] * q[2] - q[3] * q[3], 2 * (q[2] * q[3] - q[0] * q[1]),
                            2 * (q[1] * q[3] - q[0] * q[2]), 2 * (q[2] * q[3] + q[0] * q[1]),
                            q[0] * q[0] - q[1] * q[1] - q[2] * q[2] + q[3] * q[3]};
      for (int i = 0; i < 3; ++i) p[i] += Rq[3 * i] * bp[0] + Rq[3 * i + 1] * bp[1] + Rq[3 * i + 2] * bp[2];
      const double t[4] = {q[0] * bq[0] - q[1] * bq[1] - q[2] * bq[2] - q[3] * bq[3],
                           q[0] * bq[1] + q[1] * bq[0] + q[2] * bq[3] - q[3] * bq[2],
                           q[0] * bq[2] - q[1] * bq[3] + q[2] * bq[0] + q[3] * bq[1],
                           q[0] * bq[3] + q[1] * bq[2] - q[2] * bq[1] + q[3] * bq[0]};
      const double tn = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2] + t[3] * t[3]);
      for (int i = 0; i < 4; ++i) q[i] = t[i] / tn;
    }
    R[0] = q[0] * q[0] + q[1] * q[1] - q[2] * q[2] - q[3] * q[3]; R[1] = 2 * (q[1] * q[2] - q[0] * q[3]);
    R[2] = 2 * (q[1] * q[3] + q[0] * q[2]); R[3] = 2 * (q[1] * q[2] + q[0] * q[3]);
    R[4] = q[0] * q[0] - q[1] * q[1] + q[2] * q[2] - q[3] * q[3]; R[5] = 2 * (q[2] * q[3] - q[0] * q[1]);
    R[6] = 2 * (q[1] * q[3] - q[0] * q[2]); R[7] = 2 * (q[2] * q[3] + q[0] * q[1]);
    R[8] = q[0] * q[0] - q[1] * q[1] - q[2] * q[2] + q[3] * q[3];
  };
  if (d.rf_static_frame) {
    for (int blk = 0; blk < d.nrfblk; ++blk) {
      float* r = &rfblk[16 * blk];
      int body;
      std::memcpy(&body, &r[0], 4);
      double R[9], p[3];
      body_world(body, R, p);
      for (int v = 0; v < 4; ++v) {  // origin (a point), then a, b, c (directions)
        const double x[3] = {r[2 + 3 * v], r[3 + 3 * v], r[4 + 3 * v]};
        for (int i = 0; i < 3; ++i)
          r[2 + 3 * v + i] = static_cast<float>(R[3 * i] * x[0] + R[3 * i + 1] * x[1] + R[3 * i + 2] * x[2] + (v == 0 ? p[i] : 0.0));
      }
    }
  }
  P.addf(&d.rfblk, rfblk);
  // per-ray records: unit direction (z column of the site rotation) and sensordata address first
  // (one 16-byte load when the ray's pass shares body and origin), then body and origin in the body
  // frame (the world frame for static lidars)
  std::vector<float> rfray;
  for (int k = 0; k < d.nrf; ++k) {
    const int site = m.sensor_objid[rf[k]];
    const double* q = &m.site_quat[4 * site];
    double dz[3] = {2 * (q[1] * q[3] + q[0] * q[2]), 2 * (q[2] * q[3] - q[0] * q[1]),
                    q[0] * q[0] - q[1] * q[1] - q[2] * q[2] + q[3] * q[3]};
    const double n = std::sqrt(dz[0] * dz[0] + dz[1] * dz[1] + dz[2] * dz[2]);
    double dir[3] = {dz[0] / n, dz[1] / n, dz[2] / n}, org[3] = {m.site_pos[3 * site], m.site_pos[3 * site + 1], m.site_pos[3 * site + 2]};
    if (d.rf_static_frame) {
      double R[9], p[3];
      body_world(m.site_bodyid[site], R, p);
      const double d0[3] = {dir[0], dir[1], dir[2]}, o0[3] = {org[0], org[1], org[2]};
      for (int i = 0; i < 3; ++i) {
        dir[i] = R[3 * i] * d0[0] + R[3 * i + 1] * d0[1] + R[3 * i + 2] * d0[2];
        org[i] = p[i] + R[3 * i] * o0[0] + R[3 * i + 1] * o0[1] + R[3 * i + 2] * o0[2];
      }
    }
    rfray.insert(rfray.end(), {static_cast<float>(dir[0]), static_cast<float>(dir[1]), static_cast<float>(dir[2]),
                               bits(m.sensor_adr[rf[k]]), bits(m.site_bodyid[site]),
                               static_cast<float>(org[0]), static_cast<float>(org[1]), static_cast<float>(org[2])});
  }
  P.addf(&d.rfray, rfray);

  b.dblock_f = dalloc(b, P.f.size() * sizeof(float));
  b.dblock_i = dalloc(b, P.i.size() * sizeof(int));
  HIP_CHECK(hipMemcpyAsync(b.dblock_f, P.f.data(), P.f.size() * sizeof(float), hipMemcpyHostToDevice, b.stream));
  HIP_CHECK(hipMemcpyAsync(b.dblock_i, P.i.data(), P.i.size() * sizeof(int), hipMemcpyHostToDevice, b.stream));
  for (auto& kv : P.fptr) kv.first->p = static_cast<const float*>(b.dblock_f) + kv.second;
  for (auto& kv : P.iptr) kv.first->p = static_cast<const int*>(b.dblock_i) + kv.second;
  HIP_CHECK(hipStreamSynchronize(b.stream));

  // --- LDS layout (floats).  Dense mode: M and its factor as nv x nv.  Blocked mode (one env per
  // wave, G = 64): M and its factor per kinematic tree, row forces and the island scratch of the
  // sparse constraint solver.
  LdsLayout& L = b.dm.L;
  int off = 0;
  auto take = [&](int n) { int o = off; off += n; off = (off + 3) & ~3; return o; };
  const int nb = m.nbody, nj = std::max(1, m.njnt), nv = std::max(1, m.nv), ng = std::max(1, m.ngeom);
  bool want_lh = false;  // the helper waves' integrator factor (set once the helpers are decided)
  auto lds_layout = [&](bool blocked) {
    off = 0;
    L.xpos = take(3 * nb); L.xquat = take(4 * nb); L.xmat = take(9 * nb); L.xipos = take(3 * nb);
    L.xanchor = take(3 * nj); L.xaxis = take(3 * nj); L.gxpos = take(3 * ng); L.gxmat = take(9 * ng);
    L.scom = take(3 * nb); L.cinert = take(10 * nb); L.crb = d.acc_sens ? take(10 * nb) : 0; L.cdof = take(6 * nv);
    L.cdofdot = take(6 * nv); L.cvel = take(6 * nb); L.cacc = take(6 * nb); L.cfrc = take(6 * nb);
    // without accelerometer / force / torque sensors (no rne_post), crb shares cacc + cfrc (12 nb):
    // CRBA's composite inertias are dead before mj_rne starts, and mj_rne's subtree force sums
    // (6 per body at crb) overwrite only cacc, which is dead once cfrc is built
    if (!d.acc_sens) L.crb = L.cacc;
    const int msize = blocked ? std::max(1, d.nMblk) : nv * nv;
    L.M = take(msize); L.L = take(msize); L.qpos = take(std::max(1, m.nq)); L.qvel = take(nv);
    L.ctrl = take(std::max(1, m.nu)); L.qfrc_applied = take(nv); L.qacc_ws = take(nv); L.qfrc_bias = take(nv);
    L.qfrc_passive = take(nv); L.qfrc_act = take(nv); L.qfrc_smooth = take(nv); L.qacc_smooth = take(nv);
    L.qacc = take(nv + 1); L.qfrc_con = take(nv + 1);  // + a dummy word (blocked-mode solver)
    L.act_force = take(std::max(1, m.nu));
    L.ten = d.ntendon > 0 ? take(2 * d.ntendon) : 0;  // tendon lengths and velocities of the step
    L.niter = take(1);
    L.hcon = take(1);
    L.Lh = want_lh ? take(nv * nv) : 0;
    L.rfmask = take(std::max(1, d.nrfblk));
    L.trees = blocked ? take(4 * std::max(1, d.ntree)) : 0;
    L.dofb = blocked ? take(2 * nv) : 0;
    // primal solvers in blocked mode: H = M + J'DJ couples the trees a contact joins, so it is
    // stored dense (dense mode builds H in the factor slot L.L instead)
    L.H = blocked && m.solver != MRS_SOL_PGS ? take(nv * nv) : 0;
    L.Li = blocked && m.solver == MRS_SOL_PGS ? take(std::max(1, d.nMblk)) : 0;
    L.rk = m.integrator == MRS_INT_RK4 ? take(std::max(1, m.nq) + 4 * nv) : 0;
    L.total = off;
  };
  lds_layout(false);
  // static ray split: every rangefinder on a world-welded body and some ray geom on one too
  d.rf_mode = 0;
  d.rf_static_mask = 0;
  if (d.nrfblk > 0 && d.nrgeom <= 32) {
    bool static_rays = true;
    for (int k = 0; k < d.nrf; ++k)
      if (m.body_weldid[m.site_bodyid[m.sensor_objid[rf[k]]]] != 0) static_rays = false;
    for (int i = 0, g = 0; g < m.ngeom; ++g) {
      if (m.geom_rgba[4 * g + 3] == 0) continue;
      if (m.body_weldid[m.geom_bodyid[g]] == 0) d.rf_static_mask |= 1u << i;
      ++i;
    }
    if (static_rays && d.rf_static_mask && !std::getenv("MRS_NO_STATIC_RAYS")) d.rf_mode = 2;
  }
  d.rf_static = d.rf_mode ? static_cast<float*>(dalloc(b, std::max(1, d.nrf) * sizeof(float))) : nullptr;
  // workgroup-shared tables: ray-geom records, the per-ray direction + address when every ray
  // starts at one point of one body, and the rays' static hits (DevModel::shr_*)
  int shr_small = 0;
  auto layout_shared = [&]() {
    d.shr_rf = d.nrgeom * 8;
    d.shr_rfst = d.shr_rf + (d.rf_common ? 4 * d.nrf : 0);
    d.shr_blk = d.shr_rfst + (d.rf_mode == 2 ? d.nrf : 0);
    d.shr_sens = d.shr_blk + 17 * d.nrfblk;
    d.shr_fric = d.shr_sens + 16 * d.nsens_other;
    d.shr_lim = d.shr_fric + 4 * d.nfric;
    d.shr_act = d.shr_lim + 4 * d.nlim;
    d.shr_dof = d.shr_act + 20 * m.nu;
    d.shr_body = d.shr_dof + 16 * m.nv;
    d.shr_mpair = d.shr_body + 8 * m.nbody;
    d.shr_jump = d.shr_mpair + 4 * d.nMpair;
    d.shr_kbody = d.shr_jump + d.njump * m.nbody;
    d.shr_kjnt = d.shr_kbody + 25 * m.nbody;
    d.shr_kgeom = d.shr_kjnt + 13 * m.njnt;
    // the smooth-dynamics tables (from shr_act on) are staged only by lane-group kernels (G < 64);
    // blocked mode (one env per workgroup) reads them from the model block instead of paying their
    // LDS per env
    shr_small = d.shr_act;
    d.shr_total = d.shr_kgeom + 9 * m.ngeom;
    d.shr_flag = d.shr_total;  // (helper waves' signal words, one per physics wave)
    d.shr_total += 4;
  };
  layout_shared();
  // lanes per environment: the narrowest group that still gives every dof its own lane (the
  // dense M / Cholesky / PGS phases are lane-per-dof) and keeps a workgroup's LDS within 80 KB
  // (two workgroups per CU); MRS_GROUP overrides (16, 32 or 64)
  auto lds_bytes = [&](int g) {
    return (static_cast<size_t>(L.total) * envs_per_block(g) + (g == 64 ? shr_small : d.shr_total)) * sizeof(float);
  };
  // (narrow groups win even when they leave CUs idle: C4's 2048 envs run a 10-step launch in
  // 1.33 ms at G = 16 on 128 workgroups vs 4.0 ms at G = 64 on 512)
  b.group = 64;
  for (int g : {32, 16})
    if (m.nv <= g && lds_bytes(g) <= 80 * 1024) b.group = g;
  // a 16-lane model whose workgroup tables outgrow the two-per-CU budget (a dense lidar: the per-ray
  // direction table is 16 B per ray) keeps its 16-lane groups rather than dropping to 32 (~4x slower
  // on C3): the per-ray table moves out of LDS (rays read from the model block, L1/L2-resident: the
  // pass's non-common path).  MRS_G16_ONE_WG also allows one workgroup per CU (up to 160 KB)
  b.g16_one_wg = 0;
  if (b.group > 16 && m.nv <= 16) {
    if (d.rf_common) {
      // drop the common-frame ray table only if that is what lets the 16-lane layout fit; otherwise
      // the model keeps its wider groups and the table (no silent slowdown of the ray pass)
      d.rf_common = 0;
      layout_shared();
      if (lds_bytes(16) <= 80 * 1024) {
        b.group = 16;
      } else {
        d.rf_common = 1;
        layout_shared();
      }
    }
    // (one 160 KB workgroup per CU was measured slower than 32-lane groups on the mesh robot: 27 vs
    // 15 ms per 10-step launch -- a single wave per SIMD cannot hide its memory latency)
    if (b.group > 16 && lds_bytes(16) <= 160 * 1024 && std::getenv("MRS_G16_ONE_WG")) { b.group = 16; b.g16_one_wg = 1; }
  }
  if (const char* e = std::getenv("MRS_GROUP")) {
    const int g = std::atoi(e);
    if ((g == 8 || g == 16 || g == 32 || g == 64) && m.nv <= g) b.group = g;
  }
  // G = 16 with fewer waves than the device has SIMDs (C4: 2048 envs = 512 waves on 1024 SIMDs):
  // one-wave workgroups, so the waves spread over every CU instead of filling half of them four to
  // a CU (measured C4: 0.802 vs 0.822 ms per launch; C3 and C2 have a wave per SIMD or more and keep
  // four-wave workgroups -- C3's LDS tables per workgroup would cost it residency).  MRS_G16_WPB
  // overrides (1, 2 or 4)
  b.wpb16 = WavesPerBlock<16>::value;
  if (b.group == 16 && !b.g16_one_wg) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, b.device) != hipSuccess) cus = 0;
    const long waves = (static_cast<long>(b.n) * 16 + 63) / 64;
    if (cus > 0 && waves < 4L * cus) b.wpb16 = 1;
    if (const char* e = std::getenv("MRS_G16_WPB")) {
      const int w = std::atoi(e);
      if (w == 1 || w == 2 || w == 4) b.wpb16 = std::min(w, static_cast<int>(WavesPerBlock<16>::value));
    }
  }
  // extended step kernels (step.hip MRS_EXT) for models with general convex (MPR) pairs -- a pair
  // that is not plane-* and has an ellipsoid, cylinder or mesh (narrowphase's analytic routines cover
  // the rest) -- or rangefinders over more than 32 ray geoms
  b.ext = d.nrgeom > 32 && d.nrf > 0;
  for (size_t p = 0; p < b.pair_g1.size() && !b.ext; ++p) {
    const int t1 = m.geom_type[b.pair_g1[p]], t2 = m.geom_type[b.pair_g2[p]];
    auto conv = [](int t) { return t == MRS_GEOM_ELLIPSOID || t == MRS_GEOM_CYLINDER || t == MRS_GEOM_MESH; };
    if (t1 != MRS_GEOM_PLANE && t2 != MRS_GEOM_PLANE && (conv(t1) || conv(t2))) b.ext = true;
  }
  // helper waves: with one-wave workgroups (fewer waves than SIMDs, so the helpers take SIMDs that
  // would idle) every physics wave gets a second wave that runs its envs' collision pass, builds their
  // constraint rows, traces their rangefinders and factors the integrator's M + h D each step while it
  // runs the dynamics (step_kernel); models with rangefinders (<= 32 ray geoms) without RK4 and
  // without the extended kernels only.  MRS_RAY_HELPERS=0 turns them off
  {
    const char* e = std::getenv("MRS_RAY_HELPERS");
    const bool want = e ? std::atoi(e) != 0 : true;
    // (the helper kernels run at one wave per SIMD, step.hip MRS_HELPER_OCC: physics plus helper
    // waves must fit the device's SIMDs at once, i.e. at most two physics waves per CU)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, b.device) != hipSuccess) cus = 0;
    const long waves = (static_cast<long>(b.n) * 16 + 63) / 64;
    const bool fit = cus <= 0 || waves <= 2L * cus;
    b.helpers = want && fit && b.group == 16 && b.wpb16 == 1 && !b.ext && d.nrf > 0 && d.nrgeom <= 32 &&
                m.integrator != MRS_INT_RK4 && !(m.disableflags & MRS_DSBL_SENSOR) ? 1 : 0;
    // the integrator factor slot (implicit-damping Euler and implicitfast; the full implicit
    // integrator factors its own LU)
    if (b.helpers && m.integrator != MRS_INT_IMPLICIT) {
      want_lh = true;
      lds_layout(false);
    }
  }
  // the integrator's M + h D factored together with M (step.hip cholesky_ih): into M's own LDS slot
  // for PGS models, which no longer read M after the factor, into the L.Lh slot for Newton / CG
  // (their primal solve multiplies by M).  16-lane groups without helper waves (they factor it on the
  // helper), implicitfast, and no force-limited actuator (their velocity derivative depends on the
  // step's actuator forces, which come after the factor).  MRS_NO_FUSE_IH=1 factors it in integrate()
  // instead (A/B)
  {
    bool flim = false;
    for (int a = 0; a < m.nu; ++a) flim |= m.actuator_forcelimited[a] != 0;
    d.fuse_ih = b.group == 16 && !b.helpers && m.integrator == MRS_INT_IMPLICITFAST && !flim && m.nv <= 16 &&
                !std::getenv("MRS_NO_FUSE_IH") ? 1 : 0;
    if (d.fuse_ih && m.solver != MRS_SOL_PGS && !want_lh) {
      want_lh = true;
      lds_layout(false);
      if ((static_cast<size_t>(L.total) * envs_per_block(b.group, b.wpb16) + d.shr_total) * sizeof(float) > 160 * 1024) {
        d.fuse_ih = 0;  // (the extra nv x nv slot does not fit the workgroup's LDS: factor in integrate())
        want_lh = false;
        lds_layout(false);
      }
    }
  }
  d.blocked = b.group == 64 ? 1 : 0;
  if (b.group == 64) d.shr_total = shr_small;

  if (d.blocked) lds_layout(true);
  d.shr_off = L.total * envs_per_block(b.group, b.wpb16);
  if ((static_cast<size_t>(d.shr_off) + d.shr_total) * sizeof(float) > 160 * 1024)
    throw UnsupportedError("model too large for the per-environment LDS working set");
  // --- scratch layout (floats).  Dense mode: rows J and M^-1 J' as nefc x nv plus per-row scalars;
  // blocked mode: one record per row in solver order (J, M^-1 J' and dof per pipe slot, scalars)
  ScratchLayout& S = b.dm.S;
  off = 0;
  const int ne = std::max(1, d.max_efc);
  // dense rows: dense mode, and blocked mode with a primal solver (the sparse records are PGS's)
  const int dn = d.blocked && m.solver == MRS_SOL_PGS && m.cone != MRS_CONE_ELLIPTIC && d.xrows == 0 ? 0 : ne;
  S.efc_J = take(dn * nv); S.efc_MJ = take(dn * nv); S.efc_type = take(ne); S.efc_pos = take(ne);
  S.efc_margin = take(ne); S.efc_floss = take(ne); S.efc_R = take(dn); S.efc_aref = take(dn);
  S.efc_b = take(dn); S.efc_f = take(ne); S.efc_ARii = take(dn); S.con = take(kConRec * std::max(1, d.max_con));
  S.efc_rec = take(d.blocked ? ne * (2 * d.pipe_w + 12) : 0);  // step.hip RF
  S.efc_rowof = take(d.blocked ? ne : 0);
  S.efc_item = take(d.blocked ? ne : 0);
  S.efc_fq = take(d.blocked ? ne : 0);
  S.efc_hdr = take(d.blocked ? 24 * ne : 0);  // step.hip kHdr
  S.efc_quad = take(d.blocked ? 64 : 0);
  S.efc_fd = take(m.cone == MRS_CONE_ELLIPTIC && m.solver == MRS_SOL_PGS ? 2 * ne : 0);  // (16-byte aligned)
  S.stage = take(d.npair > 0 ? 64 * kMaxPairCon * 7 : 0);  // <= 64 lanes x 8 contacts x 7 floats
  S.efc_n = take(1);
  S.sens = take(std::max(1, m.nsensordata));
  S.total = off;
  b.d_dm = static_cast<DevModel*>(dalloc(b, sizeof(DevModel)));
  HIP_CHECK(hipMemcpyAsync(b.d_dm, &b.dm, sizeof(DevModel), hipMemcpyHostToDevice, b.stream));
  HIP_CHECK(hipStreamSynchronize(b.stream));
}

int field_dim(const Model& m, int field) {
  switch (field) {
    case MRS_FIELD_QPOS: return m.nq;
    case MRS_FIELD_QVEL: case MRS_FIELD_QFRC_APPLIED: case MRS_FIELD_QACC_WARMSTART: case MRS_FIELD_QACC:
    case MRS_FIELD_QFRC_ACTUATOR: return m.nv;
    case MRS_FIELD_CTRL: return m.nu;
    case MRS_FIELD_SENSORDATA: return m.nsensordata;
    case MRS_FIELD_TIME: return 1;
    case MRS_FIELD_WARNING: return 4;
    case MRS_FIELD_NCON: return 1;
    case MRS_FIELD_SOLVER_NITER: return 1;
  }
  return -1;
}
void* field_ptr(BatchImpl& b, int field) {
  switch (field) {
    case MRS_FIELD_QPOS: return b.st.qpos;
    case MRS_FIELD_QVEL: return b.st.qvel;
    case MRS_FIELD_CTRL: return b.st.ctrl;
    case MRS_FIELD_QFRC_APPLIED: return b.st.qfrc_applied;
    case MRS_FIELD_QACC_WARMSTART: return b.st.qacc_ws;
    case MRS_FIELD_QACC: return b.st.qacc;
    case MRS_FIELD_QFRC_ACTUATOR: return b.st.qfrc_act;
    case MRS_FIELD_SENSORDATA: return b.st.sensordata;
    case MRS_FIELD_TIME: return b.st.time;
    case MRS_FIELD_WARNING: return b.st.warning;
    case MRS_FIELD_NCON: return b.st.ncon;
    case MRS_FIELD_SOLVER_NITER: return b.st.niter;
  }
  return nullptr;
}

}  // namespace

BatchImpl* batch_create(const Model* model, int n_envs, int device, int max_contacts) {
  if (n_envs < 1) throw std::invalid_argument("n_envs must be positive");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) throw DeviceError("no HIP device available");
  if (device < 0 || device >= ndev) throw std::invalid_argument("device index out of range");
  HIP_CHECK(hipSetDevice(device));
  auto* b = new BatchImpl();
  try {
    b->model = model;
    b->n = n_envs;
    b->device = device;
    HIP_CHECK(hipStreamCreateWithFlags(&b->own_stream, hipStreamNonBlocking));
    b->stream = b->own_stream;
    for (int k = 0; k < 2; ++k) { HIP_CHECK(hipEventCreate(&b->ev0[k])); HIP_CHECK(hipEventCreate(&b->ev1[k])); }
    build_devmodel(*b, max_contacts);
    const Model& m = *model;
    const size_t n = static_cast<size_t>(n_envs);
    b->st.qpos = static_cast<float*>(dalloc(*b, n * std::max(1, m.nq) * sizeof(float)));
    b->st.qvel = static_cast<float*>(dalloc(*b, n * std::max(1, m.nv) * sizeof(float)));
    b->st.ctrl = static_cast<float*>(dalloc(*b, n * std::max(1, m.nu) * sizeof(float)));
    b->st.qfrc_applied = static_cast<float*>(dalloc(*b, n * std::max(1, m.nv) * sizeof(float)));
    b->st.qacc_ws = static_cast<float*>(dalloc(*b, n * std::max(1, m.nv) * sizeof(float)));
    b->st.qacc = static_cast<float*>(dalloc(*b, n * std::max(1, m.nv) * sizeof(float)));
    b->st.qfrc_act = static_cast<float*>(dalloc(*b, n * std::max(1, m.nv) * sizeof(float)));
    b->st.sensordata = static_cast<float*>(dalloc(*b, n * std::max(1, m.nsensordata) * sizeof(float)));
    b->st.time = static_cast<double*>(dalloc(*b, n * sizeof(double)));
    b->st.warning = static_cast<int*>(dalloc(*b, n * 4 * sizeof(int)));
    b->st.ncon = static_cast<int*>(dalloc(*b, n * sizeof(int)));
    b->st.niter = static_cast<int*>(dalloc(*b, n * sizeof(int)));
    // padded to whole workgroups of the chosen group width: idle groups use it
    const size_t epb = static_cast<size_t>(envs_per_block(b->group, b->wpb16));
    const size_t n_pad = (static_cast<size_t>(n) + epb - 1) / epb * epb;
    // env spread (opt-in, MRS_SPREAD=<shift>): 2^shift lane groups per env, the extra ones mirroring
    // the first, so a small batch occupies more waves.  Measured slower (round 5, same box: C4 18.2
    // vs 22.9 M env-steps/s at shift 2, C2 147 vs 156 M at shift 1): the mirrors' issue slots cost
    // more than the latency they hide, so it is off by default
    int shift = 0;
    if (const char* e = std::getenv("MRS_SPREAD")) shift = std::max(0, std::min(3, std::atoi(e)));
    const size_t n_virt = ((static_cast<size_t>(n) << shift) + epb - 1) / epb * epb;
    b->st.spread_shift = shift;
    b->st.wpb16 = b->wpb16;
    b->st.ray_helpers = b->helpers;  // (build_devmodel)
    b->st.scr_mirror = static_cast<int>(n_pad);
    b->st.scratch = static_cast<float*>(dalloc(*b, (n_pad + (shift ? n_virt : 0)) * b->S.total * sizeof(float)));
    b->st.geom_xpos = static_cast<float*>(dalloc(*b, n * std::max(1, m.ngeom) * 3 * sizeof(float)));
    b->st.geom_xmat = static_cast<float*>(dalloc(*b, n * std::max(1, m.ngeom) * 9 * sizeof(float)));
    b->st.cam_xpos = static_cast<float*>(dalloc(*b, n * std::max(1, m.ncam) * 3 * sizeof(float)));
    b->st.cam_xmat = static_cast<float*>(dalloc(*b, n * std::max(1, m.ncam) * 9 * sizeof(float)));
    batch_reset(b, -1, 0, n_envs);
    if (b->dm.rf_mode == 2) {
      // static ray hits: one forward-only pass of env 0 with the producer's model copy
      DevModel prod = b->dm;
      prod.rf_mode = 1;
      DevModel* d_prod = static_cast<DevModel*>(dalloc(*b, sizeof(DevModel)));
      HIP_CHECK(hipMemcpyAsync(d_prod, &prod, sizeof(DevModel), hipMemcpyHostToDevice, b->stream));
      HIP_CHECK(launch_step(d_prod, b->L.total, b->dm.shr_total, b->st, 1, 1, true, b->group, false, b->ext, b->stream));
      HIP_CHECK(hipStreamSynchronize(b->stream));
    }
    batch_launch(b, 1, true);  // mj_forward after load (src/mujoco_system_interface.cpp:741)
    HIP_CHECK(hipStreamSynchronize(b->stream));
  } catch (...) {
    batch_free(b);
    throw;
  }
  return b;
}

void batch_free(BatchImpl* b) {
#ifdef MRS_DEPTH_STATS
  {
    unsigned long long h[4] = {};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_depth_stats), sizeof h) == hipSuccess && h[0])
      fprintf(stderr, "depth stats: tiles %llu, candidate visits %llu (%.2f per tile), winning visits %llu (%.1f %%)\n",
              h[0], h[1], static_cast<double>(h[1]) / h[0], h[2], 100.0 * h[2] / std::max(1ull, h[1]));
  }
#endif
  if (!b) return;
  (void)hipSetDevice(b->device);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  if (b->rstream) (void)hipStreamSynchronize(b->rstream);
  for (void* p : b->allocs) (void)hipFree(p);
  if (b->rast_list) (void)hipFree(b->rast_list);
  if (b->snap_ev) (void)hipEventDestroy(b->snap_ev);
  if (b->rend_ev) (void)hipEventDestroy(b->rend_ev);
  if (b->rstream) (void)hipStreamDestroy(b->rstream);
  for (int k = 0; k < 2; ++k) {
    if (b->ev0[k]) (void)hipEventDestroy(b->ev0[k]);
    if (b->ev1[k]) (void)hipEventDestroy(b->ev1[k]);
  }
  if (b->own_stream) (void)hipStreamDestroy(b->own_stream);
  delete b;
}

int batch_num_envs(const BatchImpl* b) { return b->n; }

int batch_layout(const BatchImpl* b, int* out, int n) {
  const int v[14] = {b->group, b->dm.L.total, b->dm.S.total, b->dm.blocked, b->dm.pipe_w, b->dm.max_efc,
                     b->dm.max_con, b->dm.ntree, b->dm.shr_total, b->dm.rf_common, b->g16_one_wg,
                     b->group == 16 ? b->wpb16 : 0, b->helpers, b->dm.fuse_ih};
  int k = 0;
  for (; k < n && k < 14; ++k) out[k] = v[k];
  return k;
}

void batch_set_stream(BatchImpl* b, void* stream) {
  b->stream = stream ? static_cast<hipStream_t>(stream) : b->own_stream;
}

void batch_reset(BatchImpl* b, int key, int env0, int n) {
  const Model& m = *b->model;
  if (env0 < 0 || n < 0 || env0 + n > b->n) throw std::invalid_argument("env range out of bounds");
  if (key >= m.nkey) throw std::invalid_argument("keyframe index out of range");
  HIP_CHECK(hipSetDevice(b->device));
  std::vector<double> qpos(static_cast<size_t>(n) * m.nq), qvel(static_cast<size_t>(n) * m.nv, 0.0),
      ctrl(static_cast<size_t>(n) * m.nu, 0.0), zeros(static_cast<size_t>(n) * m.nv, 0.0), t(n, 0.0);
  for (int e = 0; e < n; ++e) {
    const double* q0 = key >= 0 ? &m.key_qpos[static_cast<size_t>(key) * m.nq] : m.qpos0.data();
    std::copy(q0, q0 + m.nq, &qpos[static_cast<size_t>(e) * m.nq]);
    if (key >= 0) {
      std::copy(&m.key_qvel[static_cast<size_t>(key) * m.nv], &m.key_qvel[static_cast<size_t>(key) * m.nv] + m.nv,
                &qvel[static_cast<size_t>(e) * m.nv]);
      std::copy(&m.key_ctrl[static_cast<size_t>(key) * m.nu], &m.key_ctrl[static_cast<size_t>(key) * m.nu] + m.nu,
                &ctrl[static_cast<size_t>(e) * m.nu]);
      t[e] = m.key_time[key];
    }
  }
  batch_set(b, MRS_FIELD_QPOS, qpos.data(), env0, n);
  batch_set(b, MRS_FIELD_QVEL, qvel.data(), env0, n);
  batch_set(b, MRS_FIELD_CTRL, ctrl.data(), env0, n);
  batch_set(b, MRS_FIELD_QFRC_APPLIED, zeros.data(), env0, n);
  batch_set(b, MRS_FIELD_QACC_WARMSTART, zeros.data(), env0, n);
  batch_set(b, MRS_FIELD_TIME, t.data(), env0, n);
  std::vector<double> w(static_cast<size_t>(n) * 4, 0.0);
  batch_set(b, MRS_FIELD_WARNING, w.data(), env0, n);
}

void batch_set(BatchImpl* b, int field, const double* host, int env0, int n) {
  const Model& m = *b->model;
  int dim = field_dim(m, field);
  if (dim < 0) throw std::invalid_argument("unknown field");
  if (env0 < 0 || n < 0 || env0 + n > b->n) throw std::invalid_argument("env range out of bounds");
  if (field == MRS_FIELD_CTRL) b->ctrl_bound = nullptr;  // (host ctrl replaces a bound buffer)
  if (n == 0 || dim == 0) return;
  HIP_CHECK(hipSetDevice(b->device));
  const size_t cnt = static_cast<size_t>(n) * dim;
  char* dst = static_cast<char*>(field_ptr(*b, field));
  if (field == MRS_FIELD_TIME) {
    HIP_CHECK(hipMemcpyAsync(dst + sizeof(double) * env0, host, cnt * sizeof(double), hipMemcpyHostToDevice, b->stream));
  } else if (field == MRS_FIELD_WARNING || field == MRS_FIELD_NCON || field == MRS_FIELD_SOLVER_NITER) {
    std::vector<int> tmp(cnt);
    for (size_t i = 0; i < cnt; ++i) tmp[i] = static_cast<int>(host[i]);
    HIP_CHECK(hipMemcpyAsync(dst + sizeof(int) * static_cast<size_t>(env0) * dim, tmp.data(), cnt * sizeof(int),
                             hipMemcpyHostToDevice, b->stream));
    HIP_CHECK(hipStreamSynchronize(b->stream));
    return;
  } else {
    std::vector<float> tmp(cnt);
    for (size_t i = 0; i < cnt; ++i) tmp[i] = static_cast<float>(host[i]);
    HIP_CHECK(hipMemcpyAsync(dst + sizeof(float) * static_cast<size_t>(env0) * dim, tmp.data(), cnt * sizeof(float),
                             hipMemcpyHostToDevice, b->stream));
    HIP_CHECK(hipStreamSynchronize(b->stream));
    return;
  }
  HIP_CHECK(hipStreamSynchronize(b->stream));
}

void batch_get(BatchImpl* b, int field, double* host, int env0, int n) {
  const Model& m = *b->model;
  int dim = field_dim(m, field);
  if (dim < 0) throw std::invalid_argument("unknown field");
  if (env0 < 0 || n < 0 || env0 + n > b->n) throw std::invalid_argument("env range out of bounds");
  if (n == 0 || dim == 0) return;
  HIP_CHECK(hipSetDevice(b->device));
  const size_t cnt = static_cast<size_t>(n) * dim;
  const char* src = field == MRS_FIELD_CTRL && b->ctrl_bound ? reinterpret_cast<const char*>(b->ctrl_bound)
                                                               : static_cast<const char*>(field_ptr(*b, field));
  if (field == MRS_FIELD_TIME) {
    HIP_CHECK(hipMemcpyAsync(host, src + sizeof(double) * env0, cnt * sizeof(double), hipMemcpyDeviceToHost, b->stream));
    HIP_CHECK(hipStreamSynchronize(b->stream));
  } else if (field == MRS_FIELD_WARNING || field == MRS_FIELD_NCON || field == MRS_FIELD_SOLVER_NITER) {
    std::vector<int> tmp(cnt);
    HIP_CHECK(hipMemcpyAsync(tmp.data(), src + sizeof(int) * static_cast<size_t>(env0) * dim, cnt * sizeof(int),
                             hipMemcpyDeviceToHost, b->stream));
    HIP_CHECK(hipStreamSynchronize(b->stream));
    for (size_t i = 0; i < cnt; ++i) host[i] = tmp[i];
  } else {
    std::vector<float> tmp(cnt);
    HIP_CHECK(hipMemcpyAsync(tmp.data(), src + sizeof(float) * static_cast<size_t>(env0) * dim, cnt * sizeof(float),
                             hipMemcpyDeviceToHost, b->stream));
    HIP_CHECK(hipStreamSynchronize(b->stream));
    for (size_t i = 0; i < cnt; ++i) host[i] = tmp[i];
  }
}

void* batch_device_ptr(BatchImpl* b, int field) { return field_ptr(*b, field); }

void batch_bind_ctrl_device(BatchImpl* b, const float* d_ctrl) { b->ctrl_bound = d_ctrl; }

void batch_set_timing(BatchImpl* b, int mask) {
  b->timing = mask;
  if (!(mask & 1)) b->ev_valid[0] = false;
  if (!(mask & 2)) b->ev_valid[1] = false;
}

void batch_set_ctrl_device(BatchImpl* b, const float* d_ctrl) {
  const Model& m = *b->model;
  b->ctrl_bound = nullptr;
  if (m.nu == 0) return;
  HIP_CHECK(hipSetDevice(b->device));
  HIP_CHECK(hipMemcpyAsync(b->st.ctrl, d_ctrl, static_cast<size_t>(b->n) * m.nu * sizeof(float),
                           hipMemcpyDeviceToDevice, b->stream));
}

void batch_launch(BatchImpl* b, int n_steps, bool forward_only) {
  if (n_steps < 1) throw std::invalid_argument("n_steps must be positive");
  HIP_CHECK(hipSetDevice(b->device));
  const bool timed = (b->timing & 1) != 0;
  if (timed) HIP_CHECK(hipEventRecord(b->ev0[0], b->stream));
  DevState st = b->st;
  if (b->ctrl_bound) st.ctrl = const_cast<float*>(b->ctrl_bound);  // (read only: loaded at launch start)
  HIP_CHECK(launch_step(b->d_dm, b->L.total, b->dm.shr_total, st, b->n, n_steps, forward_only, b->group,
                        b->model->solver != MRS_SOL_PGS, b->ext, b->stream));
  if (timed) HIP_CHECK(hipEventRecord(b->ev1[0], b->stream));
  b->ev_valid[0] = timed;
}

namespace {
struct Poses { const float *gpos, *gmat, *cpos, *cmat; };

void check_render_args(const BatchImpl* b, int cam, int env0, int n) {
  const Model& m = *b->model;
  if (cam < 0 || cam >= m.ncam) throw std::invalid_argument("camera index out of range");
  if (env0 < 0 || n < 1 || env0 + n > b->n) throw std::invalid_argument("env range out of bounds");
  if (m.ngeom > kMaxRenderGeoms) throw UnsupportedError("too many geoms for the depth kernel");
}

// depth (+ colour) kernel launch on `stream` from the given geom / camera poses, bracketed by the
// batch's render timing events
void render_launch(BatchImpl* b, int cam, int env0, int n, float* dout, unsigned char* drgb, const Poses& ps,
                   hipStream_t stream) {
  const Model& m = *b->model;
  const int W = m.cam_resolution[2 * cam], H = m.cam_resolution[2 * cam + 1];
  const float f = static_cast<float>(0.5 * H / std::tan(m.cam_fovy[cam] * M_PI / 360.0));
  const float znear = static_cast<float>(m.vis_znear * m.stat_extent), zfar = static_cast<float>(m.vis_zfar * m.stat_extent);
  const DevModel& d = b->dm;
  const MeshRef mesh{d.mesh_vert.p, d.mesh_face.p, d.geom_dataid.p, d.mesh_vertadr.p, d.mesh_faceadr.p,
                     d.mesh_facenum.p, d.mesh_bvh.p, d.mesh_bvhadr.p, d.mesh_bvhnum.p, d.mesh_tri.p};
  const LitRef lr{d.rlit.p, d.geom_matid.p, d.lit_nlight, d.lit_mat0, d.lit_tex0, d.lit_sky};
  // the binned kernel needs its band of W x kBandH 64-bit keys in LDS (within the device's per-block
  // limit) and a per-frame triangle list in global memory: frames go in chunks whose lists fit a
  // budget (MRS_RAST_BUDGET_MB, default 2048 MB), so a large mesh over many envs renders in several
  // launches instead of failing the allocation
  const size_t band_lds = static_cast<size_t>(W) * kBandH * sizeof(unsigned long long);
  if (b->max_lds == 0) {
    int v = 0;
    HIP_CHECK(hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, b->device));
    b->max_lds = v > 0 ? v : 65536;
  }
  const bool raster = d.nrast > 0 && W <= 2048 && H <= kBandH * kMaxBands && band_lds <= static_cast<size_t>(b->max_lds) &&
                     !std::getenv("MRS_DEPTH_V2") && !std::getenv("MRS_DEPTH_V1");
  const size_t per_frame = static_cast<size_t>(std::max(d.nrast_pair, 1)) * sizeof(unsigned long long);
  const char* bud = std::getenv("MRS_RAST_BUDGET_MB");
  const size_t budget = (bud ? static_cast<size_t>(std::max(1L, std::atol(bud))) : 2048) << 20;
  const int chunk = static_cast<int>(std::max<size_t>(1, std::min<size_t>(n, budget / per_frame)));
  if (raster && b->rast_frames < chunk) {
    // (one render at a time per batch: the lists are reused by every later frame batch)
    if (b->rast_list) {
      HIP_CHECK(hipStreamSynchronize(b->stream));
      if (b->rstream) HIP_CHECK(hipStreamSynchronize(b->rstream));
      HIP_CHECK(hipFree(b->rast_list));
    }
    HIP_CHECK(hipMalloc(&b->rast_list, static_cast<size_t>(chunk) * per_frame));
    b->rast_frames = chunk;
  }
  const bool timed = (b->timing & 2) != 0;
  if (timed) HIP_CHECK(hipEventRecord(b->ev0[1], stream));
  if (raster) {
    for (int c0 = 0; c0 < n; c0 += chunk) {
      const int nc = std::min(chunk, n - c0);
      const size_t px = static_cast<size_t>(c0) * W * H;
      hipLaunchKernelGGL(drgb ? depth_kernel_mesh<true> : depth_kernel_mesh<false>, dim3(nc), dim3(256), band_lds,
                         stream, d.geom_type.p, d.geom_group.p,
                         d.geom_size.p, d.geom_rgba.p, m.ngeom, ps.gpos, ps.gmat, ps.cpos, ps.cmat, m.ncam, cam,
                         env0 + c0, W, H, f, znear, zfar, dout + px, drgb ? drgb + 3 * px : nullptr, mesh,
                         d.rast_geom.p, d.rast_base.p, d.nrast, d.nrast_pair, b->rast_list, lr);
    }
  } else if (m.ngeom <= kDepthGeoms && !std::getenv("MRS_DEPTH_V1")) {
    const bool has_mesh = d.nrast > 0 || std::any_of(m.geom_type.begin(), m.geom_type.end(),
                                                      [](int t) { return t == MRS_GEOM_MESH; });
    auto kern = has_mesh ? (drgb ? depth_kernel_v2<true, true> : depth_kernel_v2<false, true>)
                         : (drgb ? depth_kernel_v2<true, false> : depth_kernel_v2<false, false>);
    hipLaunchKernelGGL(kern, dim3(n), dim3(256), 0, stream,
                       d.geom_type.p, d.geom_group.p, d.geom_size.p,
                       d.geom_rgba.p, m.ngeom, ps.gpos, ps.gmat, ps.cpos, ps.cmat, m.ncam,
                       cam, env0, W, H, f, znear, zfar, dout, drgb, mesh, lr);
  } else {
    dim3 grid(((W + 15) / 16) * ((H + 15) / 16), n);
    hipLaunchKernelGGL(drgb ? depth_kernel<true> : depth_kernel<false>, grid, dim3(256), 0, stream, d.geom_type.p,
                       d.geom_group.p, d.geom_size.p, d.geom_rbound.p,
                       d.geom_rgba.p, m.ngeom, ps.gpos, ps.gmat, ps.cpos, ps.cmat, m.ncam,
                       cam, env0, W, H, f, znear, zfar, dout, drgb, mesh, lr);
  }
  HIP_CHECK(hipGetLastError());
  if (timed) HIP_CHECK(hipEventRecord(b->ev1[1], stream));
  b->ev_valid[1] = timed;
}
}  // namespace

void batch_render_depth(BatchImpl* b, int cam, int env0, int n, float* out, bool device_out, unsigned char* rgb_out) {
  check_render_args(b, cam, env0, n);
  const Model& m = *b->model;
  HIP_CHECK(hipSetDevice(b->device));
  const int W = m.cam_resolution[2 * cam], H = m.cam_resolution[2 * cam + 1];
  const size_t bytes = static_cast<size_t>(n) * W * H * sizeof(float);
  const size_t rgb_bytes = rgb_out ? static_cast<size_t>(n) * W * H * 3 : 0;
  float* dout = out;
  unsigned char* drgb = rgb_out;
  void* tmp = nullptr;
  if (!device_out) {
    HIP_CHECK(hipMallocAsync(&tmp, bytes + rgb_bytes, b->stream));
    dout = static_cast<float*>(tmp);
    if (rgb_out) drgb = static_cast<unsigned char*>(tmp) + bytes;
  }
  if (b->rend_pending) HIP_CHECK(hipStreamWaitEvent(b->stream, b->rend_ev, 0));  // one render at a time
  render_launch(b, cam, env0, n, dout, drgb, Poses{b->st.geom_xpos, b->st.geom_xmat, b->st.cam_xpos, b->st.cam_xmat},
                b->stream);
  if (!device_out) {
    HIP_CHECK(hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, b->stream));
    if (rgb_out) HIP_CHECK(hipMemcpyAsync(rgb_out, drgb, rgb_bytes, hipMemcpyDeviceToHost, b->stream));
    HIP_CHECK(hipFreeAsync(tmp, b->stream));
    HIP_CHECK(hipStreamSynchronize(b->stream));
  }
}

// Camera pipeline: the poses of the last step are copied into a snapshot on the batch stream (so the
// copy is ordered after that step and before the next), then the frame is rendered from the snapshot
// on the batch's render stream while later steps run on the batch stream.  A new snapshot waits for
// the previous asynchronous render to finish reading the old one.  batch_render_wait orders the
// batch stream after the last render (frames complete for anything queued later).
void batch_render_async(BatchImpl* b, int cam, int env0, int n, float* d_out, unsigned char* d_rgb) {
  check_render_args(b, cam, env0, n);
  const Model& m = *b->model;
  HIP_CHECK(hipSetDevice(b->device));
  const size_t ng = static_cast<size_t>(b->n) * std::max(1, m.ngeom), nc = static_cast<size_t>(b->n) * std::max(1, m.ncam);
  if (!b->rstream) {
    HIP_CHECK(hipStreamCreateWithFlags(&b->rstream, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&b->snap_ev, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&b->rend_ev, hipEventDisableTiming));
    b->snap_gpos = static_cast<float*>(dalloc(*b, ng * 3 * sizeof(float)));
    b->snap_gmat = static_cast<float*>(dalloc(*b, ng * 9 * sizeof(float)));
    b->snap_cpos = static_cast<float*>(dalloc(*b, nc * 3 * sizeof(float)));
    b->snap_cmat = static_cast<float*>(dalloc(*b, nc * 9 * sizeof(float)));
  }
  if (b->rend_pending) HIP_CHECK(hipStreamWaitEvent(b->stream, b->rend_ev, 0));
  HIP_CHECK(hipMemcpyAsync(b->snap_gpos, b->st.geom_xpos, ng * 3 * sizeof(float), hipMemcpyDeviceToDevice, b->stream));
  HIP_CHECK(hipMemcpyAsync(b->snap_gmat, b->st.geom_xmat, ng * 9 * sizeof(float), hipMemcpyDeviceToDevice, b->stream));
  HIP_CHECK(hipMemcpyAsync(b->snap_cpos, b->st.cam_xpos, nc * 3 * sizeof(float), hipMemcpyDeviceToDevice, b->stream));
  HIP_CHECK(hipMemcpyAsync(b->snap_cmat, b->st.cam_xmat, nc * 9 * sizeof(float), hipMemcpyDeviceToDevice, b->stream));
  HIP_CHECK(hipEventRecord(b->snap_ev, b->stream));
  HIP_CHECK(hipStreamWaitEvent(b->rstream, b->snap_ev, 0));
  render_launch(b, cam, env0, n, d_out, d_rgb, Poses{b->snap_gpos, b->snap_gmat, b->snap_cpos, b->snap_cmat}, b->rstream);
  HIP_CHECK(hipEventRecord(b->rend_ev, b->rstream));
  b->rend_pending = true;
}

void batch_render_wait(BatchImpl* b) {
  HIP_CHECK(hipSetDevice(b->device));
  if (b->rend_pending) HIP_CHECK(hipStreamWaitEvent(b->stream, b->rend_ev, 0));
}

// mjData.efc_* of the last forward pass of one env (type, dense J rows, R, aref, force).  Returns
// nefc: 0 when no row was built (constraints disabled, or none active).
int batch_get_efc(BatchImpl* b, int env, int max, int* type, double* J, double* R, double* aref, double* force) {
  if (env < 0 || env >= b->n) throw std::invalid_argument("env out of bounds");
  if (max < 0) throw std::invalid_argument("negative capacity");
  if (b->dm.blocked && b->model->solver == MRS_SOL_PGS && b->model->cone != MRS_CONE_ELLIPTIC && b->dm.xrows == 0)
    throw UnsupportedError("blocked-mode PGS keeps its constraint rows in sparse records");
  HIP_CHECK(hipSetDevice(b->device));
  const ScratchLayout& S = b->S;
  const float* base = b->st.scratch + static_cast<size_t>(env) * S.total;
  int nefc = 0;
  HIP_CHECK(hipMemcpyAsync(&nefc, base + S.efc_n, sizeof(int), hipMemcpyDeviceToHost, b->stream));
  HIP_CHECK(hipStreamSynchronize(b->stream));
  if (nefc < 0) throw UnsupportedError("the register friction-loss path keeps no dense rows");
  const int n = std::min(nefc, max), nv = b->model->nv;
  if (n <= 0) return nefc;
  std::vector<float> t(n), j(static_cast<size_t>(n) * nv), r(n), a(n), f(n);
  auto get = [&](float* dst, int off, size_t count) {
    HIP_CHECK(hipMemcpyAsync(dst, base + off, count * sizeof(float), hipMemcpyDeviceToHost, b->stream));
  };
  get(t.data(), S.efc_type, n); get(j.data(), S.efc_J, j.size()); get(r.data(), S.efc_R, n);
  get(a.data(), S.efc_aref, n); get(f.data(), S.efc_f, n);
  HIP_CHECK(hipStreamSynchronize(b->stream));
  for (int i = 0; i < n; ++i) {
    int code;
    std::memcpy(&code, &t[i], sizeof code);
    if (type) type[i] = code >> 16;
    if (R) R[i] = r[i];
    if (aref) aref[i] = a[i];
    if (force) force[i] = f[i];
    if (J) for (int k = 0; k < nv; ++k) J[static_cast<size_t>(i) * nv + k] = j[static_cast<size_t>(i) * nv + k];
  }
  return nefc;
}

// mjData.contact of the last forward pass of one env (geom1/geom2 as mj_collision orders them: pair
// order g1 < g2 with the lower geom type first, then the narrow phase's order).  Records are read from
// the env's contact scratch (step.hip collision(): pair id, dist, pos, frame).  Returns ncon.
int batch_get_contacts(BatchImpl* b, int env, int max, int* geom, double* dist, double* pos, double* frame) {
  if (env < 0 || env >= b->n) throw std::invalid_argument("env out of bounds");
  if (max < 0) throw std::invalid_argument("negative capacity");
  HIP_CHECK(hipSetDevice(b->device));
  int ncon = 0;
  HIP_CHECK(hipMemcpyAsync(&ncon, b->st.ncon + env, sizeof(int), hipMemcpyDeviceToHost, b->stream));
  HIP_CHECK(hipStreamSynchronize(b->stream));
  const int n = std::min(ncon, max);
  if (n <= 0) return ncon;
  std::vector<float> rec(static_cast<size_t>(n) * kConRec);
  const float* src = b->st.scratch + static_cast<size_t>(env) * b->S.total + b->S.con;
  HIP_CHECK(hipMemcpyAsync(rec.data(), src, rec.size() * sizeof(float), hipMemcpyDeviceToHost, b->stream));
  HIP_CHECK(hipStreamSynchronize(b->stream));
  for (int c = 0; c < n; ++c) {
    const float* r = &rec[static_cast<size_t>(c) * kConRec];
    int p;
    std::memcpy(&p, r, sizeof(int));
    if (p < 0 || p >= static_cast<int>(b->pair_g1.size())) throw DeviceError("corrupt contact record");
    if (geom) { geom[2 * c] = b->pair_g1[p]; geom[2 * c + 1] = b->pair_g2[p]; }
    if (dist) dist[c] = r[1];
    if (pos) for (int i = 0; i < 3; ++i) pos[3 * c + i] = r[2 + i];
    if (frame) for (int i = 0; i < 9; ++i) frame[9 * c + i] = r[5 + i];
  }
  return ncon;
}

// fp32 field rows [env0, env0 + n) into a caller device buffer [n][dim], ordered on the batch stream
// (observation export without a host round trip, e.g. for the end-of-step RCCL gather)
void batch_get_field_device(BatchImpl* b, int field, float* d_out, int env0, int n) {
  const Model& m = *b->model;
  const int dim = field_dim(m, field);
  if (dim < 0 || field == MRS_FIELD_TIME || field == MRS_FIELD_WARNING || field == MRS_FIELD_NCON || field == MRS_FIELD_SOLVER_NITER)
    throw std::invalid_argument("not an fp32 state field");
  if (env0 < 0 || n < 0 || env0 + n > b->n) throw std::invalid_argument("env range out of bounds");
  if (n == 0 || dim == 0) return;
  HIP_CHECK(hipSetDevice(b->device));
  const float* base = field == MRS_FIELD_CTRL && b->ctrl_bound ? b->ctrl_bound
                                                               : static_cast<const float*>(field_ptr(*b, field));
  const float* src = base + static_cast<size_t>(env0) * dim;
  HIP_CHECK(hipMemcpyAsync(d_out, src, static_cast<size_t>(n) * dim * sizeof(float), hipMemcpyDeviceToDevice,
                           b->stream));
}

void batch_sync(BatchImpl* b) {
  HIP_CHECK(hipSetDevice(b->device));
  HIP_CHECK(hipStreamSynchronize(b->stream));
  if (b->rstream) HIP_CHECK(hipStreamSynchronize(b->rstream));
}

double batch_last_kernel_ms(BatchImpl* b, int kind) {
  if (kind < 0 || kind > 1 || !b->ev_valid[kind]) return -1;
  HIP_CHECK(hipSetDevice(b->device));
  HIP_CHECK(hipEventSynchronize(b->ev1[kind]));
  float ms = -1;
  if (hipEventElapsedTime(&ms, b->ev0[kind], b->ev1[kind]) != hipSuccess) return -1;
  return ms;
}

}  // namespace mrs
