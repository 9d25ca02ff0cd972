// Fused batched mj_step for CDNA4 (gfx950): one wavefront per environment.
//
// Replaces the mj_step call of the reference's physics loop (src/mujoco_system_interface.cpp:1691,
// 1731) and mj_forward (:741,1771) for N environments at once.  Each wave keeps its environment's
// kinematic/dynamic working set in LDS (layout: devmodel.h LdsLayout) for all fused steps of a
// launch; lanes work in parallel over bodies of one tree level, over geoms, dofs, mass-matrix
// entries, constraint rows, collision pairs and rangefinder rays; reductions and broadcasts use
// wavefront shuffles.  Constraint rows live in a per-env global scratch region (L2-resident).
// State in HBM is read once and written once per launch.  Pipeline stages mirror MuJoCo 3.3.4
// (see oracle/oracle.c for the fp64 restatement each stage is checked against).
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "devmodel.h"
#include "raymesh.h"

// MRS_EXT: compile the extended code paths (MPR contact polish, chunked ray pass for more than 32
// ray geoms).  The split build sets it per part (build.py); one translation unit carries them.
#ifndef MRS_EXT
#define MRS_EXT 1
#endif

namespace mrs {

namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

constexpr float kMinVal = 1e-15f;
constexpr float kMaxVal = 1e10f;

// LDS-qualified float: per-env working set pointers keep the LDS address space across the
// out-of-line phase functions, so every access is a ds_read/ds_write (not a flat access).
typedef __attribute__((address_space(3))) float lfloat;
// Global-qualified float: per-env scratch and output pointers compile to global_load/store (not flat
// accesses, which also hold the LDS counter and so stall LDS waits behind memory latency).
typedef __attribute__((address_space(1))) float gfloat;

// Phase inlining follows the register budget of the group width: with G <= 16 (2 waves/SIMD, 256
// VGPRs) every phase is inlined into the kernel (measured C3: 0.829 ms per launch vs 0.889 out of
// line, and 157 vs 384 MB of writes per launch without the callee-saved spills); at G = 64 (blocked
// mode, 3 waves/SIMD) too (C5: same speed, 4.3 GB per launch less traffic: the out-of-line phases'
// callee-saved VGPR spills, ~26 KB each way per env-step); at G = 32 phases stay out of line so each
// gets its own register allocation.  Call sites use clang's statement attributes;
// -DMRS_PHASE_INLINE / -DMRS_PHASE_OUTLINE force one policy for A/B builds.
#define MRS_PHASE
#if defined(MRS_PHASE_INLINE)
#define MRS_CALL(G, stmt) do { [[clang::always_inline]] stmt; } while (0)
#elif defined(MRS_PHASE_OUTLINE)
#define MRS_CALL(G, stmt) do { [[clang::noinline]] stmt; } while (0)
#else
#define MRS_CALL(G, stmt)                          \
  do {                                             \
    if constexpr ((G) != 32) {                     \
      [[clang::always_inline]] stmt;               \
    } else {                                       \
      [[clang::noinline]] stmt;                    \
    }                                              \
  } while (0)
#endif

// Code that is rarely executed in the fused step loop (fallbacks for trees deeper than the group):
// out of line on narrow groups, so the inlined loop the waves cycle through every step stays small
// for the instruction cache (measured C3: moving the dense constraint path out, 197 -> 137 KB of
// kernel code, took a launch from 0.716 to 0.679 ms).  Only for code whose arguments are the env
// pointers: a local array passed by address to an out-of-line call is forced into scratch memory.
#define MRS_COLD(G, stmt)                          \
  do {                                             \
    if constexpr ((G) <= 16) {                     \
      [[clang::noinline]] stmt;                    \
    } else {                                       \
      stmt;                                        \
    }                                              \
  } while (0)

// workgroup barrier between a step kernel's physics waves and their ray helper waves, which share
// only LDS (the helpers read the poses) and write disjoint sensordata words: the caller's LDS writes
// complete (lgkmcnt), and with `drain` its global stores too (vmcnt: a helper's ray results land
// before a physics wave's re-run of the step may overwrite them), then s_barrier
__device__ __forceinline__ void helper_barrier(bool drain) {
  if (drain) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// the helper wave also builds the dense constraint rows when none of them reads what the smooth
// dynamics compute (tendon rows read the step's tendon lengths from smooth_forces)
__device__ __forceinline__ bool helper_rows(const DevModel& m) { return m.ntendon == 0; }
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ float bcast(float v, int src) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}

// ---- lane groups: G consecutive lanes own one environment (64/G environments per wavefront).
// Group-local reductions, scans, broadcasts and votes; for G = 64 they are the wave-wide forms.
// DPP move within rows of 16 lanes (no LDS traffic, unlike ds_bpermute-based shuffles)
// (bound_ctrl set: every control used here reads an in-row lane, and it lets the backend fold the
// move into the consuming VALU op as a DPP source operand)
template <int kCtrl>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, 0xf, 0xf, true));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // lane i <-> 7-i within each 8
constexpr int kDppMirror = 0x140;     // lane i <-> 15-i within each 16
template <int G>
__device__ __forceinline__ float gsum(float v) {
  // full sum of each row of 16 in every lane of the row: quads, then halves, then rows.  Every lane
  // must end with the same bits (group-uniform branches and replicated solver state depend on it):
  // each step adds the same two rounded values in both lanes of a pair, which IEEE addition makes
  // symmetric -- but only if the compiler cannot contract the caller's product into the first add
  // (lane i would add its exact product to lane j's rounded one).  The empty asm makes v opaque.
  asm volatile("" : "+v"(v));
  v += dpp<kDppXor1>(v);
  v += dpp<kDppXor2>(v);
  v += dpp<kDppHalfMirror>(v);
  if constexpr (G >= 16) v += dpp<kDppMirror>(v);
  if constexpr (G >= 32) v += __shfl_xor(v, 16);
  if constexpr (G == 64) v += __shfl_xor(v, 32);
  return v;
}
// fp64 group sum (the elliptic PGS sweep's residuals): a butterfly of lane swaps within the group, so
// every lane adds the same two values and ends with the same bits (the asm keeps the caller's
// product from being contracted into the first add, as in gsum)
template <int G>
__device__ __forceinline__ double gsum_d(double v) {
  asm volatile("" : "+v"(v));
#pragma unroll
  for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o, G);
  return v;
}
template <int G>
__device__ __forceinline__ int gscan_excl(int v, int glane, int& total) {
  int x = v;
#pragma unroll
  for (int off = 1; off < G; off <<= 1) {
    int y = __shfl_up(x, off, G);
    if (glane >= off) x += y;
  }
  total = __shfl(x, G - 1, G);
  return x - v;
}
// the same exclusive group scan for small non-negative values (< 2^kBits): one ballot per bit and a
// masked lane count (v_mbcnt) -- no LDS round trips (the shuffles above are ds_bpermute chains), and
// lanes outside the exec mask count as 0
template <int G, int kBits>
__device__ __forceinline__ int gscan_excl_small(int v, int& total) {
  const int base = __lane_id() & ~(G - 1);
  const unsigned long long gmask = G == 64 ? ~0ull : (((1ull << (G & 63)) - 1) << base);
  int off = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < kBits; ++b) {
    const unsigned long long bal = __ballot((v >> b) & 1) & gmask;
    off += static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(bal >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(bal), 0u)))
           << b;
    tot += __popcll(bal) << b;
  }
  total = tot;
  return off;
}
// value of lane `src` of the caller's group, in every lane of the group: one readlane per group and
// a per-lane select (readlane reads a lane's register whatever the exec mask, and each group only
// selects its own group's value)
template <int G>
__device__ __forceinline__ float gbcast(float v, int src) {
  if constexpr (G == 64) {
    return bcast(v, src);
  } else {
    const int grp = __lane_id() / G;
    float r = bcast(v, src);
#pragma unroll
    for (int i = 1; i < 64 / G; ++i) {
      const float ri = bcast(v, src + i * G);
      r = grp == i ? ri : r;
    }
    return r;
  }
}
template <int G>
__device__ __forceinline__ bool gany(bool c) {
  if constexpr (G == 64) {
    return __any(c);
  } else {
    const unsigned long long b = __ballot(c);
    const int base = __lane_id() & ~(G - 1);
    return ((b >> base) & ((1ull << G) - 1)) != 0;
  }
}

// compile-time unrolling: f(integral_constant<int, 0..N-1>) in order
template <class F, int... K>
__device__ __forceinline__ void unroll_impl(F& f, std::integer_sequence<int, K...>) {
  (f(std::integral_constant<int, K>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void unroll(F&& f) {
  unroll_impl(f, std::make_integer_sequence<int, N>{});
}
// lane K of each row of 16 (= each group when G == 16), in every lane of the row: DPP row_newbcast
template <int K>
__device__ __forceinline__ float rowb(float v) { return dpp<0x150 + K>(v); }

// ------------------------------------------------------------------ small math (fp32)
__device__ __forceinline__ void quat_mul(float r[4], const float a[4], const float b[4]) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
__device__ __forceinline__ void quat_normalize(float q[4]) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < kMinVal) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  float in = 1.0f / n;
  q[0] *= in; q[1] *= in; q[2] *= in; q[3] *= in;
}
__device__ __forceinline__ void quat2mat(float m[9], const float q[4]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  m[0] = w * w + x * x - y * y - z * z; m[1] = 2 * (x * y - w * z); m[2] = 2 * (x * z + w * y);
  m[3] = 2 * (x * y + w * z); m[4] = w * w - x * x + y * y - z * z; m[5] = 2 * (y * z - w * x);
  m[6] = 2 * (x * z - w * y); m[7] = 2 * (y * z + w * x); m[8] = w * w - x * x - y * y + z * z;
}
__device__ __forceinline__ void mat_vec(float r[3], const float m[9], const float v[3]) {
  float a = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  float b = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  float c = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}
template <class PM>
__device__ __forceinline__ void matT_vec(float r[3], const PM* m, const float v[3]) {
  float a = m[0] * v[0] + m[3] * v[1] + m[6] * v[2];
  float b = m[1] * v[0] + m[4] * v[1] + m[7] * v[2];
  float c = m[2] * v[0] + m[5] * v[1] + m[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}
__device__ __forceinline__ void rot_quat(float r[3], const float v[3], const float q[4]) {
  float m[9];
  quat2mat(m, q);
  mat_vec(r, m, v);
}
__device__ __forceinline__ void cross3(float r[3], const float a[3], const float b[3]) {
  float x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  r[0] = x; r[1] = y; r[2] = z;
}
__device__ __forceinline__ float dot3(const float a[3], const float b[3]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ __forceinline__ float normalize3(float a[3]) {
  float n = sqrtf(dot3(a, a));
  if (n < kMinVal) { a[0] = 1; a[1] = a[2] = 0; return n; }
  float in = 1.0f / n;
  a[0] *= in; a[1] *= in; a[2] *= in;
  return n;
}
__device__ __forceinline__ void axis_angle_quat(float q[4], const float ax[3], float ang) {
  float s, c;
  sincosf(0.5f * ang, &s, &c);
  q[0] = c; q[1] = ax[0] * s; q[2] = ax[1] * s; q[3] = ax[2] * s;
}
template <class PI>
__device__ __forceinline__ void mul_inert_vec(float r[6], const PI* i, const float v[6]) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
template <class PR, class PV, class PU>
__device__ __forceinline__ void cross_motion(PR* r, const PV* v, const PU* u) {
  float t0 = -v[2] * u[1] + v[1] * u[2];
  float t1 = v[2] * u[0] - v[0] * u[2];
  float t2 = -v[1] * u[0] + v[0] * u[1];
  float t3 = -v[2] * u[4] + v[1] * u[5] - v[5] * u[1] + v[4] * u[2];
  float t4 = v[2] * u[3] - v[0] * u[5] + v[5] * u[0] - v[3] * u[2];
  float t5 = -v[1] * u[3] + v[0] * u[4] - v[4] * u[0] + v[3] * u[1];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3; r[4] = t4; r[5] = t5;
}
template <class PR, class PV, class PF>
__device__ __forceinline__ void cross_force(PR* r, const PV* v, const PF* f) {
  float t0 = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  float t1 = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  float t2 = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  float t3 = -v[2] * f[4] + v[1] * f[5];
  float t4 = v[2] * f[3] - v[0] * f[5];
  float t5 = -v[1] * f[3] + v[0] * f[4];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3; r[4] = t4; r[5] = t5;
}
__device__ __forceinline__ bool is_bad(float x) { return !(x == x) || x > kMaxVal || x < -kMaxVal; }
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// ------------------------------------------------------------------ ray primitives (engine_ray)
__device__ __forceinline__ float ray_quad(float a, float b, float c, float x[2]) {
  float det = b * b - a * c;
  if (det < kMinVal) { x[0] = x[1] = -1; return -1; }
  det = sqrtf(det);
  float ia = 1.0f / a;
  x[0] = (-b - det) * ia;
  x[1] = (-b + det) * ia;
  if (x[0] >= 0) return x[0];
  if (x[1] >= 0) return x[1];
  return -1;
}
template <class PS>
__device__ float ray_geom_local(int type, const PS s, const float lp[3], const float lv[3]) {
  float x[2];
  switch (type) {
    case MRS_GEOM_PLANE: {
      // parallel (within 1e-6 rad) or facing away: miss (fp32-safe form of MuJoCo's lv[2] > -mjMINVAL)
      if (lv[2] >= 0 || lv[2] * lv[2] <= 1e-12f * dot3(lv, lv)) return -1;
      float t = -lp[2] / lv[2];
      if (t < 0) return -1;
      float p0 = lp[0] + t * lv[0], p1 = lp[1] + t * lv[1];
      if ((s[0] <= 0 || fabsf(p0) <= s[0]) && (s[1] <= 0 || fabsf(p1) <= s[1])) return t;
      return -1;
    }
    case MRS_GEOM_SPHERE:
      return ray_quad(dot3(lv, lv), dot3(lv, lp), dot3(lp, lp) - s[0] * s[0], x);
    case MRS_GEOM_CAPSULE: {
      float best = -1;
      float a = lv[0] * lv[0] + lv[1] * lv[1];
      if (a > kMinVal) {
        float b = lv[0] * lp[0] + lv[1] * lp[1], c = lp[0] * lp[0] + lp[1] * lp[1] - s[0] * s[0];
        ray_quad(a, b, c, x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && fabsf(lp[2] + x[i] * lv[2]) <= s[1] && (best < 0 || x[i] < best)) best = x[i];
      }
      float vv = dot3(lv, lv);
      for (int e = -1; e <= 1; e += 2) {
        float q[3] = {lp[0], lp[1], lp[2] - e * s[1]};
        ray_quad(vv, dot3(lv, q), dot3(q, q) - s[0] * s[0], x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && e * (lp[2] + x[i] * lv[2] - e * s[1]) >= 0 && (best < 0 || x[i] < best)) best = x[i];
      }
      return best;
    }
    case MRS_GEOM_ELLIPSOID: {
      float q[3] = {lp[0] / s[0], lp[1] / s[1], lp[2] / s[2]}, v[3] = {lv[0] / s[0], lv[1] / s[1], lv[2] / s[2]};
      return ray_quad(dot3(v, v), dot3(v, q), dot3(q, q) - 1, x);
    }
    case MRS_GEOM_CYLINDER: {
      float best = -1;
      float a = lv[0] * lv[0] + lv[1] * lv[1];
      if (a > kMinVal) {
        float b = lv[0] * lp[0] + lv[1] * lp[1], c = lp[0] * lp[0] + lp[1] * lp[1] - s[0] * s[0];
        ray_quad(a, b, c, x);
        for (int i = 0; i < 2; ++i)
          if (x[i] >= 0 && fabsf(lp[2] + x[i] * lv[2]) <= s[1] && (best < 0 || x[i] < best)) best = x[i];
      }
      if (fabsf(lv[2]) > kMinVal)
        for (int e = -1; e <= 1; e += 2) {
          float t = (e * s[1] - lp[2]) / lv[2];
          if (t < 0) continue;
          float p0 = lp[0] + t * lv[0], p1 = lp[1] + t * lv[1];
          if (p0 * p0 + p1 * p1 <= s[0] * s[0] && (best < 0 || t < best)) best = t;
        }
      return best;
    }
    case MRS_GEOM_BOX: {
      // slab form of mj_rayBox's face test: the same face parameters (+-s - lp) / lv, nearest
      // non-negative crossing (entry from outside, exit from inside); measured C3 +5.7% over the
      // face-by-face loop (a ray grazing an edge may take the adjacent face's equal-t crossing)
      float tmin = -3.0e38f, tmax = 3.0e38f;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float inv = __builtin_amdgcn_rcpf(lv[i]);
        const bool par = fabsf(lv[i]) <= kMinVal;
        const float t1 = (-s[i] - lp[i]) * inv, t2 = (s[i] - lp[i]) * inv;
        const bool inside = fabsf(lp[i]) <= s[i];
        tmin = fmaxf(tmin, par ? (inside ? -3.0e38f : 3.0e38f) : fminf(t1, t2));
        tmax = fminf(tmax, par ? (inside ? 3.0e38f : -3.0e38f) : fmaxf(t1, t2));
      }
      if (tmax < tmin || tmax < 0) return -1;
      return tmin >= 0 ? tmin : tmax;
    }
  }
  return -1;
}

// ------------------------------------------------------------------ collision primitives
struct Con { float dist, pos[3], nrm[3]; };
typedef __attribute__((address_space(1))) Con gCon;  // narrow-phase staging lives in global scratch

__device__ __forceinline__ int sphere_sphere(const float p1[3], float r1, const float p2[3], float r2,
                                             float margin, gCon* out, int n) {
  float dv[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  float len = sqrtf(dot3(dv, dv));
  float dist = len - r1 - r2;
  if (dist > margin || n >= 4) return n;
  gCon& c = out[n];
  if (len < kMinVal) { c.nrm[0] = 1; c.nrm[1] = c.nrm[2] = 0; }
  else { float il = 1.0f / len; c.nrm[0] = dv[0] * il; c.nrm[1] = dv[1] * il; c.nrm[2] = dv[2] * il; }
  for (int i = 0; i < 3; ++i) c.pos[i] = p1[i] + c.nrm[i] * (r1 + dist / 2);
  c.dist = dist;
  return n + 1;
}
__device__ __forceinline__ void seg_point_closest(const float a[3], const float b[3], const float p[3], float c[3]) {
  float ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, ap[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
  float den = dot3(ab, ab), t = den > kMinVal ? dot3(ap, ab) / den : 0;
  t = clampf(t, 0, 1);
  for (int i = 0; i < 3; ++i) c[i] = a[i] + t * ab[i];
}
__device__ void seg_seg_closest(const float a0[3], const float a1[3], const float b0[3], const float b1[3],
                                float ca[3], float cb[3]) {
  float d1[3] = {a1[0] - a0[0], a1[1] - a0[1], a1[2] - a0[2]};
  float d2[3] = {b1[0] - b0[0], b1[1] - b0[1], b1[2] - b0[2]};
  float r[3] = {a0[0] - b0[0], a0[1] - b0[1], a0[2] - b0[2]};
  float a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  float s = 0, t = 0;
  if (a <= kMinVal && e <= kMinVal) { s = t = 0; }
  else if (a <= kMinVal) { s = 0; t = clampf(f / e, 0, 1); }
  else {
    float c = dot3(d1, r);
    if (e <= kMinVal) { t = 0; s = clampf(-c / a, 0, 1); }
    else {
      float bb = dot3(d1, d2), den = a * e - bb * bb;
      s = den > kMinVal * a * e ? clampf((bb * f - c * e) / den, 0, 1) : 0;
      t = (bb * s + f) / e;
      if (t < 0) { t = 0; s = clampf(-c / a, 0, 1); }
      else if (t > 1) { t = 1; s = clampf((bb - c) / a, 0, 1); }
    }
  }
  for (int i = 0; i < 3; ++i) { ca[i] = a0[i] + s * d1[i]; cb[i] = b0[i] + t * d2[i]; }
}
__device__ __forceinline__ int plane_sphere(const float* pp, const float* pm, const float p[3], float r,
                                            float margin, gCon* out, int n) {
  float nrm[3] = {pm[2], pm[5], pm[8]};
  float dv[3] = {p[0] - pp[0], p[1] - pp[1], p[2] - pp[2]};
  float dist = dot3(dv, nrm) - r;
  if (dist > margin || n >= 4) return n;
  gCon& c = out[n];
  for (int i = 0; i < 3; ++i) { c.pos[i] = p[i] - nrm[i] * (r + dist / 2); c.nrm[i] = nrm[i]; }
  c.dist = dist;
  return n + 1;
}
__device__ int plane_box(const float* pp, const float* pm, const float* bp, const float* bm, const float* size,
                         float margin, gCon* out, int n) {
  float nrm[3] = {pm[2], pm[5], pm[8]};
  float dv[3] = {bp[0] - pp[0], bp[1] - pp[1], bp[2] - pp[2]};
  float cdist = dot3(dv, nrm);
  for (int k = 0; k < 8 && n < 4; ++k) {
    float v[3] = {(k & 1) ? size[0] : -size[0], (k & 2) ? size[1] : -size[1], (k & 4) ? size[2] : -size[2]};
    float c[3];
    mat_vec(c, bm, v);
    float ld = dot3(nrm, c);
    float dist = cdist + ld;
    if (dist > margin || ld > 0) continue;
    gCon& o = out[n++];
    for (int i = 0; i < 3; ++i) { o.pos[i] = bp[i] + c[i] - nrm[i] * dist / 2; o.nrm[i] = nrm[i]; }
    o.dist = dist;
  }
  return n;
}
__device__ int sphere_box(const float p[3], float r, const float* bp, const float* bm, const float* size,
                          float margin, gCon* out, int n) {
  float dv[3] = {p[0] - bp[0], p[1] - bp[1], p[2] - bp[2]}, l[3];
  matT_vec(l, bm, dv);
  float c[3];
  bool inside = true;
  for (int i = 0; i < 3; ++i) {
    c[i] = clampf(l[i], -size[i], size[i]);
    if (c[i] != l[i]) inside = false;
  }
  float nl[3], dist;
  if (!inside) {
    float dl[3] = {c[0] - l[0], c[1] - l[1], c[2] - l[2]};
    float len = sqrtf(dot3(dl, dl));
    dist = len - r;
    if (dist > margin) return n;
    for (int i = 0; i < 3; ++i) nl[i] = dl[i] / len;
  } else {
    int ax = 0;
    float best = 1e30f;
    for (int i = 0; i < 3; ++i) {
      float pen = size[i] - fabsf(l[i]);
      if (pen < best) { best = pen; ax = i; }
    }
    dist = -best - r;
    nl[0] = nl[1] = nl[2] = 0;
    nl[ax] = l[ax] >= 0 ? -1.0f : 1.0f;
  }
  if (n >= 4) return n;
  gCon& o = out[n];
  float nw[3];
  mat_vec(nw, bm, nl);
  for (int i = 0; i < 3; ++i) { o.nrm[i] = nw[i]; o.pos[i] = p[i] + nw[i] * (r + dist / 2); }
  o.dist = dist;
  return n + 1;
}
// capsule (segment a-b, radius r) vs box: oracle.c col_capsule_box in fp32.  Exact closest point of the
// segment to the box (F(t), the squared box distance of the segment point, is convex and piecewise
// quadratic between the slab-crossing breakpoints: the best clamped stationary point of the pieces);
// at most 2 contacts (mjc_CapsuleBox's count): the closest point alone when it lies strictly inside
// the segment piece within the slabs of the axes where it is inside the box's extent and is clearly
// nearer than both ends of that piece (a capsule across an edge), otherwise the two ends of the piece
// (a capsule lying on a face rests on two points, where the single closest point would be arbitrary
// along the face and ill-conditioned between fp32 and fp64); a segment through the box: the point of
// deepest penetration.  Breakpoints sorted by a 19-comparator network (static registers).
__device__ __forceinline__ float seg_box_F(const float la[3], const float d[3], const float* s, float t) {
  float f = 0;
  for (int i = 0; i < 3; ++i) {
    const float e = fabsf(la[i] + t * d[i]) - s[i];
    if (e > 0) f += e * e;
  }
  return f;
}
__device__ int capsule_box(const float a[3], const float b[3], float r, const float* bp, const float* bm,
                           const float* size, float margin, gCon* out, int n) {
  float la[3], lb[3], d[3];
  {
    float da[3] = {a[0] - bp[0], a[1] - bp[1], a[2] - bp[2]}, db[3] = {b[0] - bp[0], b[1] - bp[1], b[2] - bp[2]};
    matT_vec(la, bm, da);
    matT_vec(lb, bm, db);
  }
  for (int i = 0; i < 3; ++i) d[i] = lb[i] - la[i];
  float k[8];
  k[0] = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float t = 1;
      if (fabsf(d[i]) > 1e-12f) {
        t = ((q ? size[i] : -size[i]) - la[i]) / d[i];
        if (!(t > 0 && t < 1)) t = 1;
      }
      k[1 + 2 * i + q] = t;
    }
  k[7] = 1;
  auto cs = [&](int i, int j) { const float lo = fminf(k[i], k[j]), hi = fmaxf(k[i], k[j]); k[i] = lo; k[j] = hi; };
  cs(0, 1); cs(2, 3); cs(4, 5); cs(6, 7); cs(0, 2); cs(1, 3); cs(4, 6); cs(5, 7); cs(1, 2); cs(5, 6);
  cs(0, 4); cs(3, 7); cs(1, 5); cs(2, 6); cs(1, 4); cs(3, 6); cs(2, 4); cs(3, 5); cs(3, 4);
  float tb = 0, Fb = seg_box_F(la, d, size, 0);
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    const float t0 = k[q], t1 = k[q + 1];
    if (t1 > t0) {
      const float tm = 0.5f * (t0 + t1);
      float num = 0, den = 0;
      for (int i = 0; i < 3; ++i) {
        const float x = la[i] + tm * d[i];
        if (fabsf(x) > size[i]) {
          const float sg = x > 0 ? 1.0f : -1.0f;
          num += d[i] * (la[i] - sg * size[i]);
          den += d[i] * d[i];
        }
      }
      const float t = clampf(den > 0 ? -num / den : t0, t0, t1);
      const float F = seg_box_F(la, d, size, t);
      if (F < Fb) { Fb = F; tb = t; }
    }
  }
  float p[3];
  if (Fb <= 0) {
    // the segment passes through the box: deepest point of min_i (s_i - |l_i(t)|)
    float lo = 0, hi = 1;
    for (int it = 0; it < 40; ++it) {
      const float t1 = lo + (hi - lo) / 3, t2 = hi - (hi - lo) / 3;
      float p1 = 1e30f, p2 = 1e30f;
      for (int i = 0; i < 3; ++i) {
        p1 = fminf(p1, size[i] - fabsf(la[i] + t1 * d[i]));
        p2 = fminf(p2, size[i] - fabsf(la[i] + t2 * d[i]));
      }
      if (p1 >= p2) hi = t2;
      else lo = t1;
    }
    const float t = 0.5f * (lo + hi);
    for (int i = 0; i < 3; ++i) p[i] = a[i] + t * (b[i] - a[i]);
    return sphere_box(p, r, bp, bm, size, margin, out, n);
  }
  float tc0 = 0, tc1 = 1;
  for (int j = 0; j < 3; ++j) {
    if (fabsf(la[j] + tb * d[j]) > size[j] || fabsf(d[j]) <= 1e-12f) continue;
    float u = (-size[j] - la[j]) / d[j], v = (size[j] - la[j]) / d[j];
    if (u > v) { const float x = u; u = v; v = x; }
    tc0 = fmaxf(tc0, u);
    tc1 = fminf(tc1, v);
  }
  tc0 = fminf(tc0, tb);
  tc1 = fmaxf(tc1, tb);
  const float F0 = seg_box_F(la, d, size, tc0), F1 = seg_box_F(la, d, size, tc1);
  if (tb > tc0 && tb < tc1 && sqrtf(Fb) < sqrtf(fminf(F0, F1)) - (1e-6f + 1e-4f * r)) {
    // across an edge: the closest point alone
    for (int i = 0; i < 3; ++i) p[i] = a[i] + tb * (b[i] - a[i]);
    return sphere_box(p, r, bp, bm, size, margin, out, n);
  }
  for (int i = 0; i < 3; ++i) p[i] = a[i] + tc0 * (b[i] - a[i]);
  n = sphere_box(p, r, bp, bm, size, margin, out, n);
  if (tc1 > tc0) {
    for (int i = 0; i < 3; ++i) p[i] = a[i] + tc1 * (b[i] - a[i]);
    n = sphere_box(p, r, bp, bm, size, margin, out, n);
  }
  return n;
}
__device__ __forceinline__ void capsule_ends(const float* pos, const float* mat, float hl, float a[3], float b[3]) {
  for (int i = 0; i < 3; ++i) { a[i] = pos[i] - mat[3 * i + 2] * hl; b[i] = pos[i] + mat[3 * i + 2] * hl; }
}
// box-box: the oracle's col_box_box (oracle/oracle.c) in fp32 -- separating-axis test over 15 axes
// (edge axes only when clearly better than the best face axis), face case by clipping the most
// anti-parallel face of the other box against the reference face's side planes, four deepest clipped
// vertices kept; edge case: one contact between the support edges.  Out of line: rare, and its
// clipping slots stay out of the hot path's registers.
// Templated on the group width only so each kernel instantiation gets its own copy, compiled under
// that kernel's register budget (a shared callee is allocated for the widest caller)
// The poses are read from the env's LDS and the sizes from the model here, not passed as arrays: a
// caller array whose address escapes into a call lives in scratch, and the caller's pair loop would
// store every pair's pose there whether or not it reaches this function.
// row i (0..2, runtime) of a 3x3 register matrix / element i of a 3-vector, by selects: a runtime
// index into a private array would place the array in scratch memory
__device__ __forceinline__ void row3_sel(const float M[3][3], int i, float out[3]) {
  for (int c = 0; c < 3; ++c) out[c] = i == 0 ? M[0][c] : (i == 1 ? M[1][c] : M[2][c]);
}
__device__ __forceinline__ float elt3_sel(const float v[3], int i) { return i == 0 ? v[0] : (i == 1 ? v[1] : v[2]); }

template <int G>
__device__ int box_box(const lfloat* gxpos, const lfloat* gxmat, CPtr<float> gsize, int g1, int g2,
                                    float margin, gCon* out) {
  float p1[3], p2[3], h1[3], h2[3], A[3][3], B[3][3];
  for (int i = 0; i < 3; ++i) {
    p1[i] = gxpos[3 * g1 + i]; p2[i] = gxpos[3 * g2 + i];
    h1[i] = gsize[3 * g1 + i]; h2[i] = gsize[3 * g2 + i];
    for (int c = 0; c < 3; ++c) { A[i][c] = gxmat[9 * g1 + 3 * c + i]; B[i][c] = gxmat[9 * g2 + 3 * c + i]; }
  }
  float d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  float best_face = -1e30f, best_edge = -1e30f, nf[3] = {0, 0, 0}, ne[3] = {0, 0, 0};
  int face_axis = -1, edge_i = -1, edge_j = -1;
  // a later face axis must beat the best by more than `tie` (oracle.c col_box_box): resting faces have
  // equal separations along both boxes' normals, and rounding must not pick the reference face
  const float tie = 1e-5f * (h1[0] + h1[1] + h1[2] + h2[0] + h2[1] + h2[2]);
  // the 15 axes unrolled (every matrix index compile-time: the boxes' frames stay in registers); a
  // separating axis is remembered and ends the test after the loop -- the same answer as leaving at it
  bool separated = false;
  unroll<15>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    float L[3];
    if constexpr (k < 3) { L[0] = A[k][0]; L[1] = A[k][1]; L[2] = A[k][2]; }
    else if constexpr (k < 6) { L[0] = B[k - 3][0]; L[1] = B[k - 3][1]; L[2] = B[k - 3][2]; }
    else cross3(L, A[(k - 6) / 3], B[(k - 6) % 3]);
    const float ln = sqrtf(dot3(L, L));
    if (ln >= 1e-6f) {
      for (int c = 0; c < 3; ++c) L[c] /= ln;
      float ra = 0, rb = 0;
      for (int i = 0; i < 3; ++i) { ra += h1[i] * fabsf(dot3(A[i], L)); rb += h2[i] * fabsf(dot3(B[i], L)); }
      const float sv = dot3(d, L);
      const float sep = fabsf(sv) - ra - rb;
      separated |= sep > margin;
      const float sg = sv >= 0 ? 1.0f : -1.0f;
      if constexpr (k < 6) {
        if (sep > best_face + tie) { best_face = sep; face_axis = k; for (int c = 0; c < 3; ++c) nf[c] = sg * L[c]; }
      } else if (sep > best_edge) {
        best_edge = sep; edge_i = (k - 6) / 3; edge_j = (k - 6) % 3;
        for (int c = 0; c < 3; ++c) ne[c] = sg * L[c];
      }
    }
  });
  if (separated || face_axis < 0) return 0;
  if (edge_i >= 0 && best_edge > best_face + 0.05f * fabsf(best_face) + 1e-6f) {
    float a0[3], a1[3], b0[3], b1[3], c1[3], c2[3], Ae[3], Be[3];
    row3_sel(A, edge_i, Ae);
    row3_sel(B, edge_j, Be);
    const float hae = elt3_sel(h1, edge_i), hbe = elt3_sel(h2, edge_j);
    for (int c = 0; c < 3; ++c) { a0[c] = p1[c]; b0[c] = p2[c]; }
    for (int i = 0; i < 3; ++i) {
      if (i != edge_i) {
        const float sg = dot3(A[i], ne) >= 0 ? 1.0f : -1.0f;
        for (int c = 0; c < 3; ++c) a0[c] += sg * h1[i] * A[i][c];
      }
      if (i != edge_j) {
        const float sg = dot3(B[i], ne) >= 0 ? -1.0f : 1.0f;
        for (int c = 0; c < 3; ++c) b0[c] += sg * h2[i] * B[i][c];
      }
    }
    for (int c = 0; c < 3; ++c) {
      a1[c] = a0[c] + hae * Ae[c]; a0[c] -= hae * Ae[c];
      b1[c] = b0[c] + hbe * Be[c]; b0[c] -= hbe * Be[c];
    }
    seg_seg_closest(a0, a1, b0, b1, c1, c2);
    gCon& o = out[0];
    for (int c = 0; c < 3; ++c) { o.pos[c] = 0.5f * (c1[c] + c2[c]); o.nrm[c] = ne[c]; }
    o.dist = best_edge;
    return 1;
  }
  // face case: reference box r (normal nr pointing at the other box), incident box i (register
  // copies chosen by selects)
  const bool refA = face_axis < 3;
  const int ir = refA ? face_axis : face_axis - 3;
  float pr[3], pi[3], hr[3], hi[3], Rr[3][3], Ri[3][3], nr[3];
  for (int c = 0; c < 3; ++c) {
    pr[c] = refA ? p1[c] : p2[c]; pi[c] = refA ? p2[c] : p1[c];
    hr[c] = refA ? h1[c] : h2[c]; hi[c] = refA ? h2[c] : h1[c];
    nr[c] = refA ? nf[c] : -nf[c];
    for (int e = 0; e < 3; ++e) { Rr[c][e] = refA ? A[c][e] : B[c][e]; Ri[c][e] = refA ? B[c][e] : A[c][e]; }
  }
  int j = 0;
  float bestc = -1;
  for (int k = 0; k < 3; ++k) {
    const float cc = fabsf(dot3(Ri[k], nr));
    if (cc > bestc) { bestc = cc; j = k; }
  }
  const int k1 = (j + 1) % 3, k2 = (j + 2) % 3;
  float Rij[3], Rik1[3], Rik2[3];
  row3_sel(Ri, j, Rij); row3_sel(Ri, k1, Rik1); row3_sel(Ri, k2, Rik2);
  const float hij = elt3_sel(hi, j), hik1 = elt3_sel(hi, k1), hik2 = elt3_sel(hi, k2);
  const float sgn = dot3(Rij, nr) > 0 ? -1.0f : 1.0f;
  // Clipping in the reference face's frame: u, v along its in-plane axes Rr[r1], Rr[r2] and w along
  // nr, measured from the face centre cr, so the four side planes are |u| <= hr[r1], |v| <= hr[r2]
  // and a vertex's separation is w.  Sutherland-Hodgman with the polygon in 8 static register slots:
  // each side emits, in input order, every vertex inside and every edge crossing, and output slot o
  // takes the candidate whose running count is o (no private-memory arrays: a scratch round trip per
  // vertex made this the slowest part of the contact-rich step).
  const int r1 = (ir + 1) % 3, r2 = (ir + 2) % 3;
  float Rr1[3], Rr2[3];
  row3_sel(Rr, r1, Rr1); row3_sel(Rr, r2, Rr2);
  const float hr0 = elt3_sel(hr, ir), hr1 = elt3_sel(hr, r1), hr2 = elt3_sel(hr, r2);
  float cr[3];
  for (int c = 0; c < 3; ++c) cr[c] = pr[c] + hr0 * nr[c];
  float pu[8], pv[8], pw[8];
  for (int vtx = 0; vtx < 4; ++vtx) {
    const float su = (vtx == 0 || vtx == 3) ? 1.0f : -1.0f, sv = (vtx < 2) ? 1.0f : -1.0f;
    float q[3];
    for (int c = 0; c < 3; ++c)
      q[c] = pi[c] + sgn * hij * Rij[c] + su * hik1 * Rik1[c] + sv * hik2 * Rik2[c] - cr[c];
    pu[vtx] = dot3(q, Rr1); pv[vtx] = dot3(q, Rr2); pw[vtx] = dot3(q, nr);
  }
  for (int vtx = 4; vtx < 8; ++vtx) { pu[vtx] = 0; pv[vtx] = 0; pw[vtx] = 0; }
  int np = 4;
#pragma unroll
  for (int side = 0; side < 4; ++side) {
    const float lim = (side < 2) ? hr1 : hr2;
    const float sg = (side & 1) ? -1.0f : 1.0f;
    float f[8];
#pragma unroll
    for (int vtx = 0; vtx < 8; ++vtx) f[vtx] = sg * (side < 2 ? pu[vtx] : pv[vtx]) - lim;
    float qu[8], qv[8], qw[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) { qu[o] = 0; qv[o] = 0; qw[o] = 0; }
    int cnt = 0;
#pragma unroll
    for (int vtx = 0; vtx < 8; ++vtx) {
      const bool in = vtx < np;
      const bool wrap = vtx + 1 >= np;
      const int nx = vtx + 1 < 8 ? vtx + 1 : 0;
      const float fa = f[vtx], fb = wrap ? f[0] : f[nx];
      const float bu = wrap ? pu[0] : pu[nx], bv = wrap ? pv[0] : pv[nx], bw = wrap ? pw[0] : pw[nx];
      const bool ea = in && fa <= 0;
      const bool ei = in && ((fa < 0 && fb > 0) || (fa > 0 && fb < 0));
      const float t = ei ? fa / (fa - fb) : 0.0f;
      const float iu = pu[vtx] + t * (bu - pu[vtx]), iv = pv[vtx] + t * (bv - pv[vtx]), iw = pw[vtx] + t * (bw - pw[vtx]);
      const int pa = cnt, pb = cnt + (ea ? 1 : 0);
#pragma unroll
      for (int o = 0; o < 8; ++o) {
        if (ea && pa == o) { qu[o] = pu[vtx]; qv[o] = pv[vtx]; qw[o] = pw[vtx]; }
        if (ei && pb == o) { qu[o] = iu; qv[o] = iv; qw[o] = iw; }
      }
      cnt = pb + (ei ? 1 : 0);
    }
    np = cnt < 8 ? cnt : 8;
#pragma unroll
    for (int o = 0; o < 8; ++o) { pu[o] = qu[o]; pv[o] = qv[o]; pw[o] = qw[o]; }
    if (np == 0) return 0;
  }
  // every clipped vertex within the margin, in clip order (up to 8; oracle.c col_box_box): choosing
  // the deepest few would decide among the equal depths of two flat-resting faces by rounding
  int n = 0;
#pragma unroll
  for (int vtx = 0; vtx < 8; ++vtx) {
    if (vtx < np && pw[vtx] <= margin) {
      const float bu = pu[vtx], bv = pv[vtx], bs = pw[vtx];
      gCon& o = out[n++];
      for (int c = 0; c < 3; ++c) {
        const float pt = cr[c] + bu * Rr1[c] + bv * Rr2[c] + bs * nr[c];
        o.pos[c] = pt - nr[c] * bs / 2;
        o.nrm[c] = nf[c];
      }
      o.dist = bs;
    }
  }
  return n;
}

// ---- general convex pairs (ellipsoid, cylinder, mesh): Minkowski Portal Refinement in fp32, the
// same steps as the oracle's mpr_penetration (oracle.c; MuJoCo mjc_Convex via libccd's
// ccdMPRPenetration with each shape inflated by margin/2, mpr_tolerance 1e-6, 50 iterations).  One
// contact: dist = margin - depth, normal geom1 -> geom2, position midway between the shapes'
// portal-interpolated surface points.  Lane-parallel like every narrow-phase routine (one pair per
// lane); mesh hull vertices are read from the model block (per-lane global loads).
constexpr float kMprTol = 1e-6f, kMprEps = 1e-10f;
constexpr int kMprIter = 50;
struct Shape {
  int type, vadr, hadr, nhull;
  float pos[3], mat[9], size[3], inflate;
};
struct MprPoint { float v[3], a[3], b[3]; };
struct MeshTab { CPtr<float> vert; CPtr<int> hull; };  // the model's mesh vertices and hull ids

__device__ __forceinline__ void shape_support(const MeshTab m, const Shape& s, const float dir[3], float out[3]) {
  float l[3], p[3] = {0, 0, 0};
  matT_vec(l, s.mat, dir);
  const float* z = s.size;
  switch (s.type) {
    case MRS_GEOM_SPHERE:
    case MRS_GEOM_CAPSULE: {
      const float n = sqrtf(dot3(l, l));
      if (n > kMinVal) for (int i = 0; i < 3; ++i) p[i] = z[0] * l[i] / n;
      if (s.type == MRS_GEOM_CAPSULE) p[2] += l[2] >= 0 ? z[1] : -z[1];
      break;
    }
    case MRS_GEOM_ELLIPSOID: {
      const float t[3] = {z[0] * z[0] * l[0], z[1] * z[1] * l[1], z[2] * z[2] * l[2]};
      const float den = sqrtf(t[0] * l[0] + t[1] * l[1] + t[2] * l[2]);
      if (den > kMinVal) for (int i = 0; i < 3; ++i) p[i] = t[i] / den;
      break;
    }
    case MRS_GEOM_CYLINDER: {
      const float rr = sqrtf(l[0] * l[0] + l[1] * l[1]);
      if (rr > kMinVal) { p[0] = z[0] * l[0] / rr; p[1] = z[0] * l[1] / rr; }
      p[2] = l[2] >= 0 ? z[1] : -z[1];
      break;
    }
    case MRS_GEOM_BOX:
      for (int i = 0; i < 3; ++i) p[i] = l[i] >= 0 ? z[i] : -z[i];
      break;
    case MRS_GEOM_MESH: {
      float best = -3.0e38f;
      for (int k = 0; k < s.nhull; ++k) {
        const int v = 3 * (s.vadr + m.hull[s.hadr + k]);
        const float x = m.vert[v], y = m.vert[v + 1], w = m.vert[v + 2];
        const float d = x * l[0] + y * l[1] + w * l[2];
        if (d > best) { best = d; p[0] = x; p[1] = y; p[2] = w; }
      }
      break;
    }
    default: break;
  }
  mat_vec(out, s.mat, p);
  const float dn = sqrtf(dot3(dir, dir));
  const float k = dn > kMinVal ? s.inflate / dn : 0.0f;
  for (int i = 0; i < 3; ++i) out[i] += s.pos[i] + k * dir[i];
}
__device__ __forceinline__ void mpr_support(const MeshTab m, const Shape& A, const Shape& B, const float dir[3],
                                            MprPoint& p) {
  const float nd[3] = {-dir[0], -dir[1], -dir[2]};
  shape_support(m, A, dir, p.a);
  shape_support(m, B, nd, p.b);
  for (int i = 0; i < 3; ++i) p.v[i] = p.a[i] - p.b[i];
}
__device__ __forceinline__ void tri_normal(float n[3], const float a[3], const float b[3], const float c[3]) {
  const float u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, v[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  cross3(n, u, v);
  normalize3(n);
}
// closest point to the origin on triangle abc (Ericson 5.1.5)
__device__ __forceinline__ void closest_on_triangle(const float a[3], const float b[3], const float c[3], float out[3]) {
  float ab[3], ac[3], ap[3], bp[3], cp[3];
  for (int i = 0; i < 3; ++i) {
    ab[i] = b[i] - a[i]; ac[i] = c[i] - a[i];
    ap[i] = -a[i]; bp[i] = -b[i]; cp[i] = -c[i];
  }
  const float d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) { for (int i = 0; i < 3; ++i) out[i] = a[i]; return; }
  const float d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { for (int i = 0; i < 3; ++i) out[i] = b[i]; return; }
  const float vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    const float t = d1 / (d1 - d3);
    for (int i = 0; i < 3; ++i) out[i] = a[i] + t * ab[i];
    return;
  }
  const float d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) { for (int i = 0; i < 3; ++i) out[i] = c[i]; return; }
  const float vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    const float t = d2 / (d2 - d6);
    for (int i = 0; i < 3; ++i) out[i] = a[i] + t * ac[i];
    return;
  }
  const float va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    const float t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int i = 0; i < 3; ++i) out[i] = b[i] + t * (c[i] - b[i]);
    return;
  }
  const float den = 1.0f / (va + vb + vc), v = vb * den, w = vc * den;
  for (int i = 0; i < 3; ++i) out[i] = a[i] + ab[i] * v + ac[i] * w;
}
// MPR's penetration vector: the point of the final portal nearest the origin.  When the origin's
// projection onto the portal plane falls inside the portal (the usual end: the origin ray crosses it)
// that point is depth * n with n the portal normal and depth = n.p1 -- well conditioned even for a
// long thin portal, whose barycentric closest-point formula cancels catastrophically in fp32 (a 0.3 m
// portal 0.07 mm from the origin: fp32 put the point on the wrong edge, 1.1 rad off).  Otherwise the
// nearest edge / vertex point (closest_on_triangle).  oracle.c mpr_nearest takes the same branches.
__device__ __forceinline__ void mpr_nearest(const float a[3], const float b[3], const float c[3], float out[3]) {
  float n[3];
  tri_normal(n, a, b, c);
  const float d = dot3(n, a);
  const float q[3] = {d * n[0], d * n[1], d * n[2]};
  // inside: q on the inner side of each edge (sign of (e x (q - v)).n, edges in winding order)
  auto side = [&](const float* u, const float* v) {
    const float e[3] = {v[0] - u[0], v[1] - u[1], v[2] - u[2]}, w[3] = {q[0] - u[0], q[1] - u[1], q[2] - u[2]};
    float x[3];
    cross3(x, e, w);
    return dot3(x, n);
  };
  if (side(a, b) >= 0 && side(b, c) >= 0 && side(c, a) >= 0) {
    for (int i = 0; i < 3; ++i) out[i] = q[i];
    return;
  }
  closest_on_triangle(a, b, c, out);
}
__device__ __forceinline__ void mpr_expand(MprPoint p[4], const MprPoint& v4) {
  float x[3];
  cross3(x, v4.v, p[0].v);
  if (dot3(p[1].v, x) > 0) {
    if (dot3(p[2].v, x) > 0) p[1] = v4;
    else p[3] = v4;
  } else {
    if (dot3(p[3].v, x) > 0) p[2] = v4;
    else p[1] = v4;
  }
}
__device__ __forceinline__ bool mpr_reach_tolerance(const MprPoint p[4], const MprPoint& v4, const float n[3]) {
  const float d4 = dot3(v4.v, n);
  const float g = fminf(d4 - dot3(p[1].v, n), fminf(d4 - dot3(p[2].v, n), d4 - dot3(p[3].v, n)));
  return g <= kMprTol;
}
// 0: origin inside the portal cone, 1: touching, 2: origin on segment p0-p1, -1: separated
__device__ __forceinline__ int mpr_discover(const MeshTab m, const Shape& A, const Shape& B, MprPoint p[4]) {
  for (int i = 0; i < 3; ++i) { p[0].a[i] = A.pos[i]; p[0].b[i] = B.pos[i]; p[0].v[i] = A.pos[i] - B.pos[i]; }
  if (dot3(p[0].v, p[0].v) < 1e-20f) p[0].v[0] += 1e-5f;
  float dir[3] = {-p[0].v[0], -p[0].v[1], -p[0].v[2]};
  normalize3(dir);
  mpr_support(m, A, B, dir, p[1]);
  if (dot3(p[1].v, dir) <= 0) return -1;
  cross3(dir, p[0].v, p[1].v);
  if (dot3(dir, dir) < kMprEps) return dot3(p[1].v, p[1].v) < kMprEps ? 1 : 2;
  normalize3(dir);
  mpr_support(m, A, B, dir, p[2]);
  if (dot3(p[2].v, dir) <= 0) return -1;
  float va[3], vb[3];
  for (int i = 0; i < 3; ++i) { va[i] = p[1].v[i] - p[0].v[i]; vb[i] = p[2].v[i] - p[0].v[i]; }
  cross3(dir, va, vb);
  normalize3(dir);
  if (dot3(dir, p[0].v) > 0) {
    const MprPoint t = p[1];
    p[1] = p[2];
    p[2] = t;
    for (int i = 0; i < 3; ++i) dir[i] = -dir[i];
  }
  for (int it = 0; it < kMprIter; ++it) {
    mpr_support(m, A, B, dir, p[3]);
    if (dot3(p[3].v, dir) <= 0) return -1;
    float x[3];
    bool replaced = false;
    cross3(x, p[1].v, p[3].v);
    if (dot3(x, p[0].v) < -kMprEps) { p[2] = p[3]; replaced = true; }
    else {
      cross3(x, p[3].v, p[2].v);
      if (dot3(x, p[0].v) < -kMprEps) { p[1] = p[3]; replaced = true; }
    }
    if (!replaced) return 0;
    for (int i = 0; i < 3; ++i) { va[i] = p[1].v[i] - p[0].v[i]; vb[i] = p[2].v[i] - p[0].v[i]; }
    cross3(dir, va, vb);
    normalize3(dir);
  }
  return 0;
}
__device__ __forceinline__ void mpr_position(const MprPoint p[4], float pos[3]) {
  float n[3], x[3], b[4];
  tri_normal(n, p[1].v, p[2].v, p[3].v);
  cross3(x, p[1].v, p[2].v); b[0] = dot3(x, p[3].v);
  cross3(x, p[3].v, p[2].v); b[1] = dot3(x, p[0].v);
  cross3(x, p[0].v, p[1].v); b[2] = dot3(x, p[3].v);
  cross3(x, p[2].v, p[1].v); b[3] = dot3(x, p[0].v);
  float sum = b[0] + b[1] + b[2] + b[3];
  if (sum <= kMprEps) {
    b[0] = 0;
    cross3(x, p[2].v, p[3].v); b[1] = dot3(x, n);
    cross3(x, p[3].v, p[1].v); b[2] = dot3(x, n);
    cross3(x, p[1].v, p[2].v); b[3] = dot3(x, n);
    sum = b[1] + b[2] + b[3];
  }
  for (int i = 0; i < 3; ++i) {
    float pa = 0, pb = 0;
    for (int k = 0; k < 4; ++k) { pa += b[k] * p[k].a[i]; pb += b[k] * p[k].b[i]; }
    pos[i] = 0.5f * (pa + pb) / sum;
  }
}
// inlined: as an out-of-line call its ABI raised the G = 32 / 64 kernels from 128 / 168 VGPRs to
// 246 (half the occupancy) for every model; inlined it only adds scratch to the convex path
__device__ __forceinline__ bool mpr_penetration(const MeshTab m, const Shape A, const Shape B,
                                                          float& depth, float nrm[3], float pos[3]) {
  MprPoint p[4], v4;
  const int r = mpr_discover(m, A, B, p);
  if (r < 0 || r == 1) return false;
  if (r == 2) {
    for (int i = 0; i < 3; ++i) { nrm[i] = p[1].v[i]; pos[i] = 0.5f * (p[1].a[i] + p[1].b[i]); }
    depth = normalize3(nrm);
    return true;
  }
  for (int it = 0;; ++it) {
    float n[3];
    tri_normal(n, p[1].v, p[2].v, p[3].v);
    if (dot3(n, p[1].v) >= 0) break;
    mpr_support(m, A, B, n, v4);
    if (dot3(v4.v, n) < 0 || mpr_reach_tolerance(p, v4, n) || it >= kMprIter) return false;
    mpr_expand(p, v4);
  }
  for (int it = 0;; ++it) {
    float n[3];
    tri_normal(n, p[1].v, p[2].v, p[3].v);
    mpr_support(m, A, B, n, v4);
    if (mpr_reach_tolerance(p, v4, n) || it > kMprIter) {
      mpr_nearest(p[1].v, p[2].v, p[3].v, nrm);
      depth = sqrtf(dot3(nrm, nrm));
      if (depth < kMinVal) return false;
      for (int i = 0; i < 3; ++i) nrm[i] /= depth;
      mpr_position(p, pos);
      return true;
    }
    mpr_expand(p, v4);
  }
}
// MPR contact polish (oracle.c mpr_polish, same steps in fp32): the minimiser over unit n of the
// support function of A - B next to MPR's normal, by active-set Newton over the shapes' polyhedral
// features (vertex / edge / face) with the smooth parts' curvature; MPR's contact is kept for pairs
// without a curved shape, cylinders, and iterations that do not settle.
constexpr int kPolMaxV = 4, kPolPasses = 12, kPolNewton = 12;
struct PolPart {
  int nv, mesh, ell, vadr, hadr;
  float v[8][3];
  float pos[3], mat[9];
  float sgn, R, M[9];
};
__device__ __forceinline__ bool pol_part_of(const Shape& s, float sgn, PolPart& p) {
  p.sgn = sgn; p.R = s.inflate; p.mesh = 0; p.ell = 0; p.nv = 0; p.vadr = s.vadr; p.hadr = s.hadr;
  for (int i = 0; i < 3; ++i) p.pos[i] = s.pos[i];
  for (int i = 0; i < 9; ++i) { p.mat[i] = s.mat[i]; p.M[i] = 0; }
  const float* z = s.size;
  switch (s.type) {
    case MRS_GEOM_SPHERE:
      p.nv = 1; p.R += z[0];
      for (int i = 0; i < 3; ++i) p.v[0][i] = sgn * s.pos[i];
      return true;
    case MRS_GEOM_CAPSULE:
      p.nv = 2; p.R += z[0];
      for (int i = 0; i < 3; ++i) {
        p.v[0][i] = sgn * (s.pos[i] - s.mat[3 * i + 2] * z[1]);
        p.v[1][i] = sgn * (s.pos[i] + s.mat[3 * i + 2] * z[1]);
      }
      return true;
    case MRS_GEOM_ELLIPSOID:
      p.nv = 1; p.ell = 1;
      for (int i = 0; i < 3; ++i) p.v[0][i] = sgn * s.pos[i];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          float v = 0;
          for (int k = 0; k < 3; ++k) v += s.mat[3 * i + k] * z[k] * z[k] * s.mat[3 * j + k];
          p.M[3 * i + j] = v;
        }
      return true;
    case MRS_GEOM_BOX:
      p.nv = 8;
      for (int k = 0; k < 8; ++k) {
        const float l[3] = {(k & 1) ? z[0] : -z[0], (k & 2) ? z[1] : -z[1], (k & 4) ? z[2] : -z[2]};
        float x[3];
        mat_vec(x, s.mat, l);
        for (int i = 0; i < 3; ++i) p.v[k][i] = sgn * (s.pos[i] + x[i]);
      }
      return true;
    case MRS_GEOM_MESH:
      p.nv = s.nhull; p.mesh = 1;
      return true;
    default:
      return false;
  }
}
__device__ __forceinline__ void pol_vertex(const MeshTab mt, const PolPart& p, int k, float out[3]) {
  if (!p.mesh) { for (int i = 0; i < 3; ++i) out[i] = p.v[k][i]; return; }
  const int v = 3 * (p.vadr + mt.hull[p.hadr + k]);
  const float l[3] = {mt.vert[v], mt.vert[v + 1], mt.vert[v + 2]};
  float x[3];
  mat_vec(x, p.mat, l);
  for (int i = 0; i < 3; ++i) out[i] = p.sgn * (p.pos[i] + x[i]);
}
__device__ __forceinline__ void pol_smooth(const PolPart& p, const float n[3], float s[3], float H[9]) {
  for (int i = 0; i < 3; ++i) s[i] = p.R * n[i];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) H[3 * i + j] += p.R * ((i == j ? 1.0f : 0.0f) - n[i] * n[j]);
  if (p.ell) {
    float Mn[3];
    mat_vec(Mn, p.M, n);
    const float h = sqrtf(dot3(n, Mn));
    if (h < kMinVal) return;
    for (int i = 0; i < 3; ++i) s[i] += Mn[i] / h;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) H[3 * i + j] += (p.M[3 * i + j] - Mn[i] * Mn[j] / (h * h)) / h;
  }
}
struct PolState { int F[2][kPolMaxV], nf[2]; };
__device__ __forceinline__ void pol_grad(const MeshTab mt, const PolPart* P, const PolState& st, const float n[3], float G[3],
                                         float H[9], float sS[2][3]) {
  for (int i = 0; i < 9; ++i) H[i] = 0;
  for (int i = 0; i < 3; ++i) G[i] = 0;
  for (int q = 0; q < 2; ++q) {
    float v0[3];
    pol_smooth(P[q], n, sS[q], H);
    pol_vertex(mt, P[q], st.F[q][0], v0);
    for (int i = 0; i < 3; ++i) G[i] += sS[q][i] + v0[i];
  }
}
__device__ __forceinline__ int pol_basis(const MeshTab mt, const PolPart* P, const PolState& st, float Q[3][3]) {
  int r = 0;
  for (int q = 0; q < 2; ++q) {
    float v0[3];
    pol_vertex(mt, P[q], st.F[q][0], v0);
    for (int k = 1; k < st.nf[q]; ++k) {
      float e[3];
      pol_vertex(mt, P[q], st.F[q][k], e);
      for (int i = 0; i < 3; ++i) e[i] -= v0[i];
      const float len = sqrtf(dot3(e, e));
      for (int j = 0; j < r; ++j) {
        const float d = dot3(e, Q[j]);
        for (int i = 0; i < 3; ++i) e[i] -= d * Q[j][i];
      }
      const float el = sqrtf(dot3(e, e));
      if (el <= 1e-5f * len || len < kMinVal) continue;
      if (r == 3) return 4;
      for (int i = 0; i < 3; ++i) Q[r][i] = e[i] / el;
      ++r;
    }
  }
  return r;
}
__device__ __forceinline__ void pol_tangent(const float n[3], float t1[3], float t2[3]) {
  float a[3] = {0, 0, 0};
  a[fabsf(n[0]) < 0.6f ? 0 : (fabsf(n[1]) < 0.6f ? 1 : 2)] = 1;
  const float d = dot3(a, n);
  for (int i = 0; i < 3; ++i) t1[i] = a[i] - d * n[i];
  normalize3(t1);
  cross3(t2, n, t1);
}
__device__ __forceinline__ int pol_move(const MeshTab mt, const PolPart* P, PolState& st, float n[3], const float dl[3]) {
  float tmin = 1;
  int qmin = -1, kmin = -1;
  for (int q = 0; q < 2; ++q) {
    float v0[3];
    pol_vertex(mt, P[q], st.F[q][0], v0);
    const float c0 = dot3(v0, n), d0 = dot3(v0, dl);
    for (int k = 0; k < P[q].nv; ++k) {
      bool in = false;
      for (int f = 0; f < st.nf[q]; ++f) in |= st.F[q][f] == k;
      if (in) continue;
      float v[3];
      pol_vertex(mt, P[q], k, v);
      const float c = dot3(v, n) - c0, d = dot3(v, dl) - d0;
      if (c + d <= 0 || d <= 0) continue;
      const float t = fmaxf(-c / d, 0.0f);
      if (t < tmin) { tmin = t; qmin = q; kmin = k; }
    }
  }
  for (int i = 0; i < 3; ++i) n[i] += tmin * dl[i];
  normalize3(n);
  if (qmin < 0) return 0;
  if (st.nf[qmin] >= kPolMaxV) return -1;
  st.F[qmin][st.nf[qmin]++] = kmin;
  return 1;
}
__device__ __forceinline__ void pol_drop(PolState& st, int q, int f) {
  for (int k = f; k + 1 < st.nf[q]; ++k) st.F[q][k] = st.F[q][k + 1];
  --st.nf[q];
}
__device__ __forceinline__ float det3(const float A[9]) {
  return A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) + A[2] * (A[3] * A[7] - A[4] * A[6]);
}
__device__ int pol_kkt(const MeshTab mt, const PolPart* P, PolState& st, const float n[3], const float G[3],
                       float w[2][kPolMaxV]) {
  float t1[3], t2[3];
  pol_tangent(n, t1, t2);
  const int m = st.nf[0] + st.nf[1] - 2;
  for (int q = 0; q < 2; ++q)
    for (int f = 0; f < kPolMaxV; ++f) w[q][f] = 0;
  if (m == 0) return 1;
  float E[6][2];
  int cq[6], cf[6], nc = 0;
  for (int q = 0; q < 2; ++q) {
    float v0[3];
    pol_vertex(mt, P[q], st.F[q][0], v0);
    for (int f = 1; f < st.nf[q]; ++f) {
      float e[3];
      pol_vertex(mt, P[q], st.F[q][f], e);
      for (int i = 0; i < 3; ++i) e[i] -= v0[i];
      E[nc][0] = dot3(e, t1); E[nc][1] = dot3(e, t2);
      cq[nc] = q; cf[nc] = f; ++nc;
    }
  }
  const float g1 = dot3(G, t1), g2 = dot3(G, t2);
  if (m == 1) {
    const float el2 = E[0][0] * E[0][0] + E[0][1] * E[0][1];
    if (el2 < kMinVal) return -1;
    const float x = -(g1 * E[0][0] + g2 * E[0][1]) / el2;
    if (x < 0) { pol_drop(st, cq[0], cf[0]); return 0; }
    if (x > 1) { pol_drop(st, cq[0], 0); return 0; }
    w[cq[0]][cf[0]] = x;
    return 1;
  }
  if (m == 2) {
    const float det = E[0][0] * E[1][1] - E[1][0] * E[0][1];
    if (fabsf(det) < kMinVal) return -1;
    const float x0 = (-g1 * E[1][1] + g2 * E[1][0]) / det, x1 = (-g2 * E[0][0] + g1 * E[0][1]) / det;
    if (cq[0] == cq[1]) {
      const float x2 = 1 - x0 - x1, worst = fminf(x2, fminf(x0, x1));
      if (worst < 0) { pol_drop(st, cq[0], worst == x0 ? cf[0] : (worst == x1 ? cf[1] : 0)); return 0; }
    } else {
      const float v0 = fminf(x0, 1 - x0), v1 = fminf(x1, 1 - x1);
      if (v0 < 0 || v1 < 0) {
        const int c = v0 <= v1 ? 0 : 1;
        const float x = c == 0 ? x0 : x1;
        pol_drop(st, cq[c], x < 0 ? cf[c] : 0);
        return 0;
      }
    }
    w[cq[0]][cf[0]] = x0;
    w[cq[1]][cf[1]] = x1;
    return 1;
  }
  if (m == 3 && (st.nf[0] == 1 || st.nf[1] == 1)) {
    const int q = cq[0];
    for (int a = 0; a < 3; ++a)
      for (int b = a + 1; b < 3; ++b) {
        const float det = E[a][0] * E[b][1] - E[b][0] * E[a][1];
        if (fabsf(det) < kMinVal) continue;
        const float x0 = (-g1 * E[b][1] + g2 * E[b][0]) / det, x1 = (-g2 * E[a][0] + g1 * E[a][1]) / det;
        if (x0 >= 0 && x1 >= 0 && x0 + x1 <= 1) { w[q][cf[a]] = x0; w[q][cf[b]] = x1; return 1; }
      }
    const float A3[9] = {E[0][0], E[1][0], E[2][0], E[0][1], E[1][1], E[2][1], 1, 1, 1}, rhs[3] = {-g1, -g2, 1};
    const float dA = det3(A3);
    if (fabsf(dA) > kMinVal) {
      float x[3];
      for (int c = 0; c < 3; ++c) {
        float B3[9];
        for (int i = 0; i < 9; ++i) B3[i] = A3[i];
        for (int r = 0; r < 3; ++r) B3[3 * r + c] = rhs[r];
        x[c] = det3(B3) / dA;
      }
      if (x[0] >= 0 && x[1] >= 0 && x[2] >= 0) {
        w[q][cf[0]] = x[0]; w[q][cf[1]] = x[1]; w[q][cf[2]] = x[2];
        return 1;
      }
    }
    return -1;
  }
  return -1;
}
// returns true with the polished depth / normal / position, false to keep MPR's
__device__ bool mpr_polish(const MeshTab mt, const Shape& A, const Shape& B, const float n0[3], float mpr_depth,
                           float& depth, float nrm[3], float pos[3]) {
  if (A.type == MRS_GEOM_CYLINDER || B.type == MRS_GEOM_CYLINDER) return false;
  const bool curvedA = A.type == MRS_GEOM_SPHERE || A.type == MRS_GEOM_CAPSULE || A.type == MRS_GEOM_ELLIPSOID;
  const bool curvedB = B.type == MRS_GEOM_SPHERE || B.type == MRS_GEOM_CAPSULE || B.type == MRS_GEOM_ELLIPSOID;
  if (!curvedA && !curvedB) return false;
  PolPart P[2];
  if (!pol_part_of(A, 1.0f, P[0]) || !pol_part_of(B, -1.0f, P[1])) return false;
  PolState st;
  float n[3] = {n0[0], n0[1], n0[2]};
  for (int q = 0; q < 2; ++q) {
    float best = -3.0e38f;
    st.nf[q] = 1;
    st.F[q][0] = 0;
    for (int k = 0; k < P[q].nv; ++k) {
      float v[3];
      pol_vertex(mt, P[q], k, v);
      const float d = dot3(v, n);
      if (d > best) { best = d; st.F[q][0] = k; }
    }
  }
  float G[3], H[9], sS[2][3], w[2][kPolMaxV];
  bool done = false;
  for (int pass = 0; pass < kPolPasses && !done; ++pass) {
    float Q[3][3];
    const int rank = pol_basis(mt, P, st, Q);
    if (rank > 2) {
      pol_grad(mt, P, st, n, G, H, sS);
      bool found = false;
      for (int q = 0; q < 2 && !found; ++q)
        for (int f = 0; f < st.nf[q] && !found; ++f) {
          PolState t = st;
          pol_drop(t, q, f);
          float Qt[3][3];
          if (pol_basis(mt, P, t, Qt) != 2) continue;
          float Gt[3], Ht[9], sSt[2][3];
          pol_grad(mt, P, t, n, Gt, Ht, sSt);
          if (pol_kkt(mt, P, t, n, Gt, w) == 1) {
            st = t;
            found = true;
            for (int i = 0; i < 3; ++i) { G[i] = Gt[i]; sS[0][i] = sSt[0][i]; sS[1][i] = sSt[1][i]; }
          }
        }
      if (!found) return false;
      done = true;
      break;
    }
    bool moved = false, conv = false;
    if (rank == 2) {
      float t[3], dl[3];
      cross3(t, Q[0], Q[1]);
      normalize3(t);
      if (dot3(t, n) < 0) for (int i = 0; i < 3; ++i) t[i] = -t[i];
      for (int i = 0; i < 3; ++i) dl[i] = t[i] - n[i];
      const int r = pol_move(mt, P, st, n, dl);
      if (r < 0) return false;
      moved = r > 0;
      conv = r == 0;
    } else {
      for (int it = 0; it < kPolNewton; ++it) {
        float dl[3];
        if (rank == 0) {
          pol_grad(mt, P, st, n, G, H, sS);
          const float lam = dot3(G, n);
          float t1[3], t2[3], Ht1[3], Ht2[3];
          pol_tangent(n, t1, t2);
          mat_vec(Ht1, H, t1);
          mat_vec(Ht2, H, t2);
          const float a11 = dot3(t1, Ht1) - lam, a22 = dot3(t2, Ht2) - lam, a12 = dot3(t1, Ht2);
          const float det = a11 * a22 - a12 * a12;
          if (!(a11 > 0 && det > 0)) return false;
          const float b1 = -dot3(G, t1), b2 = -dot3(G, t2);
          const float x1 = (b1 * a22 - b2 * a12) / det, x2 = (b2 * a11 - b1 * a12) / det;
          for (int i = 0; i < 3; ++i) dl[i] = x1 * t1[i] + x2 * t2[i];
        } else {
          const float d = dot3(n, Q[0]);
          for (int i = 0; i < 3; ++i) n[i] -= d * Q[0][i];
          normalize3(n);
          pol_grad(mt, P, st, n, G, H, sS);
          const float lm = dot3(G, n);
          float t[3], Ht[3];
          cross3(t, Q[0], n);
          mat_vec(Ht, H, t);
          const float f2 = dot3(t, Ht) - lm;
          if (!(f2 > 0)) return false;
          const float th = -dot3(G, t) / f2;
          for (int i = 0; i < 3; ++i) dl[i] = th * t[i];
        }
        const float step = sqrtf(dot3(dl, dl));
        const int r = pol_move(mt, P, st, n, dl);
        if (r < 0) return false;
        if (r > 0) { moved = true; break; }
        // (fp32: a step below 2e-6 leaves an error of order its square, under the rounding floor)
        if (step < 2e-6f) { conv = true; break; }
      }
    }
    if (moved) continue;
    if (!conv) return false;
    pol_grad(mt, P, st, n, G, H, sS);
    const int k = pol_kkt(mt, P, st, n, G, w);
    if (k < 0) return false;
    done = k == 1;
  }
  if (!done) return false;
  const float dp = dot3(G, n);
  if (dot3(n, n0) < 0.8f || !(dp > 0) || dp > mpr_depth + kMprTol) return false;
  float pA[3], pB[3];
  for (int q = 0; q < 2; ++q) {
    float* pt = q ? pB : pA;
    float v0[3];
    pol_vertex(mt, P[q], st.F[q][0], v0);
    for (int i = 0; i < 3; ++i) pt[i] = v0[i] + sS[q][i];
    for (int f = 1; f < st.nf[q]; ++f) {
      float e[3];
      pol_vertex(mt, P[q], st.F[q][f], e);
      for (int i = 0; i < 3; ++i) pt[i] += w[q][f] * (e[i] - v0[i]);
    }
  }
  depth = dp;
  for (int i = 0; i < 3; ++i) { nrm[i] = n[i]; pos[i] = 0.5f * (pA[i] - pB[i]); }
  return true;
}
__device__ __forceinline__ void shape_of(const DevModel& m, int g, const float* p, const float* mat, const float* size,
                                         float inflate, Shape& s) {
  s.type = m.geom_type[g];
  for (int i = 0; i < 3; ++i) { s.pos[i] = p[i]; s.size[i] = size[i]; }
  for (int i = 0; i < 9; ++i) s.mat[i] = mat[i];
  s.inflate = inflate;
  s.vadr = s.hadr = s.nhull = 0;
  if (s.type == MRS_GEOM_MESH) {
    const int id = m.geom_dataid[g];
    s.vadr = m.mesh_vertadr[id];
    s.hadr = m.mesh_hulladr[id];
    s.nhull = m.mesh_hullnum[id];
  }
}
#if MRS_EXT
// face contacts of two polytopes (box and mesh pairs, at least one mesh; oracle.c col_poly_faces
// restates the same steps in fp64): the support faces along MPR's normal, and when
// the better aligned one is within kPolyCos of it, the other face's polygon clipped by its side
// planes, every clipped vertex within margin of the reference plane a contact (at most
// kMaxPairCon).  Returns -1 when the pair is not face-on or a support face has more than kPolyMaxV
// vertices (MPR's single contact stays).  Inlined: out of line, its reference arguments forced the
// caller's model copy and shapes into scratch memory, which cost the mesh robot's extended kernel
// 10 % (C3m 4.42 -> 4.84 ms per launch) although that scene has no polytope pair.
constexpr int kPolyMaxV = 8;
constexpr float kPolyCos = 0.999f;
struct PolyFace { int n; float v[kPolyMaxV][3]; float nrm[3]; };
__device__ __forceinline__ float poly_support_face(const DevModel& m, const Shape& s, int g, const float dir[3],
                                                   PolyFace& f) {
  const float* R = s.mat;
  if (s.type == MRS_GEOM_BOX) {
    float l[3];
    for (int i = 0; i < 3; ++i) l[i] = R[i] * dir[0] + R[3 + i] * dir[1] + R[6 + i] * dir[2];
    int ax = 0;
    for (int i = 1; i < 3; ++i)
      if (fabsf(l[i]) > fabsf(l[ax])) ax = i;
    const float sg = l[ax] >= 0 ? 1.0f : -1.0f;
    const int j = (ax + 1) % 3, k = (ax + 2) % 3;
    const float cj[4] = {-1, 1, 1, -1}, ck[4] = {-1, -1, 1, 1};
    f.n = 4;
    for (int q = 0; q < 4; ++q) {
      const int qq = sg > 0 ? q : 3 - q;
      float lp[3];
      lp[ax] = sg * s.size[ax];
      lp[j] = cj[qq] * s.size[j];
      lp[k] = ck[qq] * s.size[k];
      for (int i = 0; i < 3; ++i) f.v[q][i] = s.pos[i] + (R[3 * i] * lp[0] + R[3 * i + 1] * lp[1] + R[3 * i + 2] * lp[2]);
    }
    for (int i = 0; i < 3; ++i) f.nrm[i] = sg * R[3 * i + ax];
    return fabsf(l[ax]);
  }
  const int id = m.geom_dataid[g];
  int best = -1;
  float ba = -3;
  const int q0 = m.mesh_polyadr[id], q1 = q0 + m.mesh_polynum[id];
  for (int q = q0; q < q1; ++q) {
    const float nl[3] = {m.mesh_polynormal[3 * q], m.mesh_polynormal[3 * q + 1], m.mesh_polynormal[3 * q + 2]};
    float a = 0;
    for (int i = 0; i < 3; ++i) a += (R[3 * i] * nl[0] + R[3 * i + 1] * nl[1] + R[3 * i + 2] * nl[2]) * dir[i];
    if (a > ba) { ba = a; best = q; }
  }
  if (best < 0 || m.mesh_polyvertnum[best] > kPolyMaxV) return -2;
  const float nl[3] = {m.mesh_polynormal[3 * best], m.mesh_polynormal[3 * best + 1], m.mesh_polynormal[3 * best + 2]};
  for (int i = 0; i < 3; ++i) f.nrm[i] = R[3 * i] * nl[0] + R[3 * i + 1] * nl[1] + R[3 * i + 2] * nl[2];
  f.n = m.mesh_polyvertnum[best];
  const int va = m.mesh_vertadr[id], pa = m.mesh_polyvertadr[best];
  for (int q = 0; q < f.n; ++q) {
    const int vi = va + m.mesh_polyvert[pa + q];
    const float lp[3] = {m.mesh_vert[3 * vi], m.mesh_vert[3 * vi + 1], m.mesh_vert[3 * vi + 2]};
    for (int i = 0; i < 3; ++i) f.v[q][i] = s.pos[i] + (R[3 * i] * lp[0] + R[3 * i + 1] * lp[1] + R[3 * i + 2] * lp[2]);
  }
  return ba;
}
__device__ __forceinline__ int poly_face_contacts(const DevModel& m, const Shape& A, int g1, const Shape& B,
                                                            int g2, const float nrm[3], float margin, gCon* out) {
  PolyFace fa, fb;
  const float nb[3] = {-nrm[0], -nrm[1], -nrm[2]};
  const float aa = poly_support_face(m, A, g1, nrm, fa), ab = poly_support_face(m, B, g2, nb, fb);
  if (aa < -1 || ab < -1) return -1;
  const bool refA = !(ab > aa + 1e-4f);
  if ((refA ? aa : ab) < kPolyCos) return -1;
  const PolyFace& ref = refA ? fa : fb;
  const PolyFace& inc = refA ? fb : fa;
  float buf[2][2 * kPolyMaxV][3];
  int cnt = inc.n, cur = 0;
  for (int q = 0; q < cnt; ++q)
    for (int i = 0; i < 3; ++i) buf[0][q][i] = inc.v[q][i];
  for (int e = 0; e < ref.n && cnt > 0; ++e) {
    const float* r0 = ref.v[e];
    const float* r1 = ref.v[(e + 1) % ref.n];
    const float ed[3] = {r1[0] - r0[0], r1[1] - r0[1], r1[2] - r0[2]};
    float h[3];
    cross3(h, ref.nrm, ed);
    int on = 0;
    for (int q = 0; q < cnt; ++q) {
      const float* pc = buf[cur][q];
      const float* pn = buf[cur][(q + 1) % cnt];
      const float dc = (pc[0] - r0[0]) * h[0] + (pc[1] - r0[1]) * h[1] + (pc[2] - r0[2]) * h[2];
      const float dn = (pn[0] - r0[0]) * h[0] + (pn[1] - r0[1]) * h[1] + (pn[2] - r0[2]) * h[2];
      if (dc >= 0 && on < 2 * kPolyMaxV)
        for (int i = 0; i < 3; ++i) buf[1 - cur][on][i] = pc[i];
      if (dc >= 0) ++on;
      if ((dc >= 0) != (dn >= 0) && on < 2 * kPolyMaxV) {
        const float t = dc / (dc - dn);
        for (int i = 0; i < 3; ++i) buf[1 - cur][on][i] = pc[i] + t * (pn[i] - pc[i]);
        ++on;
      }
    }
    cnt = on < 2 * kPolyMaxV ? on : 2 * kPolyMaxV;
    cur = 1 - cur;
  }
  const float sg = refA ? 1.0f : -1.0f;
  int n = 0;
  for (int q = 0; q < cnt && n < kMaxPairCon; ++q) {
    const float* p = buf[cur][q];
    const float d = (p[0] - ref.v[0][0]) * ref.nrm[0] + (p[1] - ref.v[0][1]) * ref.nrm[1] + (p[2] - ref.v[0][2]) * ref.nrm[2];
    if (d > margin) continue;
    gCon& o = out[n++];
    for (int i = 0; i < 3; ++i) { o.pos[i] = p[i] - 0.5f * d * ref.nrm[i]; o.nrm[i] = sg * ref.nrm[i]; }
    o.dist = d;
  }
  return n > 0 ? n : -1;
}
#endif
__device__ __forceinline__ int convex_convex(const DevModel& m, int g1, int g2, const float* p1, const float* m1, const float* s1,
                             const float* p2, const float* m2, const float* s2, float margin, gCon* out) {
  Shape A, B;
  shape_of(m, g1, p1, m1, s1, 0.5f * margin, A);
  shape_of(m, g2, p2, m2, s2, 0.5f * margin, B);
  float depth, nrm[3], pos[3];
  if (!mpr_penetration(MeshTab{m.mesh_vert, m.mesh_hull}, A, B, depth, nrm, pos)) return 0;
#if MRS_EXT
  {
    // two polytopes, at least one a mesh: the face contacts when the contact is face-on
    const bool p1 = A.type == MRS_GEOM_BOX || A.type == MRS_GEOM_MESH, p2 = B.type == MRS_GEOM_BOX || B.type == MRS_GEOM_MESH;
    if (p1 && p2 && (A.type == MRS_GEOM_MESH || B.type == MRS_GEOM_MESH) && !(m.restate & MRS_RESTATE_NO_MULTICCD)) {
      const int r = poly_face_contacts(m, A, g1, B, g2, nrm, margin, out);
      if (r >= 0) return r;
    }
  }
#endif
#if MRS_EXT
  if (!(m.restate & MRS_RESTATE_NO_MPR_POLISH)) {
    const float n0[3] = {nrm[0], nrm[1], nrm[2]};
    [[clang::noinline]] mpr_polish(MeshTab{m.mesh_vert, m.mesh_hull}, A, B, n0, depth, depth, nrm, pos);
  }
#endif
  gCon& o = out[0];
  for (int i = 0; i < 3; ++i) { o.pos[i] = pos[i]; o.nrm[i] = nrm[i]; }
  o.dist = margin - depth;
  return 1;
}
// plane (geom1) vs ellipsoid: the support point along -normal
__device__ __forceinline__ int plane_support(const DevModel& m, int g2, const float* pp, const float* pm, const float* p2,
                             const float* m2, const float* s2, float margin, gCon* out) {
  Shape B;
  shape_of(m, g2, p2, m2, s2, 0.0f, B);
  const float nrm[3] = {pm[2], pm[5], pm[8]}, nd[3] = {-nrm[0], -nrm[1], -nrm[2]};
  float s[3];
  shape_support(MeshTab{m.mesh_vert, m.mesh_hull}, B, nd, s);
  const float dv[3] = {s[0] - pp[0], s[1] - pp[1], s[2] - pp[2]};
  const float dist = dot3(dv, nrm);
  if (dist > margin) return 0;
  gCon& o = out[0];
  for (int i = 0; i < 3; ++i) { o.pos[i] = s[i] - nrm[i] * dist / 2; o.nrm[i] = nrm[i]; }
  o.dist = dist;
  return 1;
}
// plane vs cylinder (oracle.c col_plane_cylinder): deepest rim point of each cap, plus the rim points
// at +-120 degrees on the deeper cap; the rim direction falls back to the cylinder's x axis when the
// axis is parallel to the normal
__device__ int plane_cylinder(const float* pp, const float* pm, const float* cp, const float* cm, const float* size,
                              float margin, gCon* out) {
  const float nrm[3] = {pm[2], pm[5], pm[8]}, ax[3] = {cm[2], cm[5], cm[8]};
  const float an = dot3(ax, nrm);
  float d[3];
  for (int i = 0; i < 3; ++i) d[i] = -nrm[i] + an * ax[i];
  if (dot3(d, d) < 1e-12f) { d[0] = cm[0]; d[1] = cm[3]; d[2] = cm[6]; }
  normalize3(d);
  float e[3];
  cross3(e, ax, d);
  const float sdeep = an > 0 ? -1.0f : 1.0f;
  int n = 0;
  for (int cap = 0; cap < 2; ++cap) {
    const float sc = cap == 0 ? sdeep : -sdeep;
    const int npts = cap == 0 ? 3 : 1;
    for (int k = 0; k < npts; ++k) {
      const float cu = k == 0 ? 1.0f : -0.5f, cv = k == 0 ? 0.0f : (k == 1 ? 0.8660254037844386f : -0.8660254037844386f);
      float p[3], dv[3];
      for (int i = 0; i < 3; ++i) p[i] = cp[i] + sc * size[1] * ax[i] + size[0] * (cu * d[i] + cv * e[i]);
      for (int i = 0; i < 3; ++i) dv[i] = p[i] - pp[i];
      const float dist = dot3(dv, nrm);
      if (dist > margin) continue;
      gCon& o = out[n++];
      for (int i = 0; i < 3; ++i) { o.pos[i] = p[i] - nrm[i] * dist / 2; o.nrm[i] = nrm[i]; }
      o.dist = dist;
    }
  }
  return n;
}
// plane vs mesh: every convex-hull vertex within margin, in hull order (at most kMaxPairCon)
__device__ __forceinline__ int plane_mesh(const DevModel& m, int g2, const float* pp, const float* pm, const float* bp,
                          const float* bm, float margin, gCon* out) {
  const float nrm[3] = {pm[2], pm[5], pm[8]};
  const int id = m.geom_dataid[g2];
  const int vadr = m.mesh_vertadr[id], hadr = m.mesh_hulladr[id], nh = m.mesh_hullnum[id];
  int n = 0;
  for (int k = 0; k < nh && n < kMaxPairCon; ++k) {
    const int v = 3 * (vadr + m.mesh_hull[hadr + k]);
    const float lv[3] = {m.mesh_vert[v], m.mesh_vert[v + 1], m.mesh_vert[v + 2]};
    float p[3];
    mat_vec(p, bm, lv);
    for (int i = 0; i < 3; ++i) p[i] += bp[i];
    const float dv[3] = {p[0] - pp[0], p[1] - pp[1], p[2] - pp[2]};
    const float dist = dot3(dv, nrm);
    if (dist > margin) continue;
    gCon& o = out[n++];
    for (int i = 0; i < 3; ++i) { o.pos[i] = p[i] - nrm[i] * dist / 2; o.nrm[i] = nrm[i]; }
    o.dist = dist;
  }
  return n;
}

template <int G>
__device__ int narrowphase(const DevModel& m, int t1, int t2, const float* p1, const float* m1, const float* s1,
                           const float* p2, const float* m2, const float* s2, float margin, gCon* out,
                           const lfloat* gxpos, const lfloat* gxmat, CPtr<float> gsize, int g1, int g2) {
  float a1[3], b1[3], a2[3], b2[3], c1[3], c2[3];
  int n = 0;
  if (t1 == MRS_GEOM_PLANE) {
    if (t2 == MRS_GEOM_SPHERE) return plane_sphere(p1, m1, p2, s2[0], margin, out, 0);
    if (t2 == MRS_GEOM_CAPSULE) {
      capsule_ends(p2, m2, s2[1], a2, b2);
      n = plane_sphere(p1, m1, a2, s2[0], margin, out, 0);
      return plane_sphere(p1, m1, b2, s2[0], margin, out, n);
    }
    if (t2 == MRS_GEOM_BOX) return plane_box(p1, m1, p2, m2, s2, margin, out, 0);
    if (t2 == MRS_GEOM_ELLIPSOID) return plane_support(m, g2, p1, m1, p2, m2, s2, margin, out);
    if (t2 == MRS_GEOM_CYLINDER) return plane_cylinder(p1, m1, p2, m2, s2, margin, out);
    if (t2 == MRS_GEOM_MESH) return plane_mesh(m, g2, p1, m1, p2, m2, margin, out);
    return 0;
  } else if (t1 == MRS_GEOM_SPHERE) {
    if (t2 == MRS_GEOM_SPHERE) return sphere_sphere(p1, s1[0], p2, s2[0], margin, out, 0);
    if (t2 == MRS_GEOM_CAPSULE) {
      capsule_ends(p2, m2, s2[1], a2, b2);
      seg_point_closest(a2, b2, p1, c2);
      return sphere_sphere(p1, s1[0], c2, s2[0], margin, out, 0);
    }
    if (t2 == MRS_GEOM_BOX) return sphere_box(p1, s1[0], p2, m2, s2, margin, out, 0);
  } else if (t1 == MRS_GEOM_CAPSULE) {
    if (t2 == MRS_GEOM_CAPSULE) {
      capsule_ends(p1, m1, s1[1], a1, b1);
      capsule_ends(p2, m2, s2[1], a2, b2);
      seg_seg_closest(a1, b1, a2, b2, c1, c2);
      return sphere_sphere(c1, s1[0], c2, s2[0], margin, out, 0);
    }
    if (t2 == MRS_GEOM_BOX) {
      capsule_ends(p1, m1, s1[1], a1, b1);
      return capsule_box(a1, b1, s1[0], p2, m2, s2, margin, out, 0);
    }
  } else if (t1 == MRS_GEOM_BOX && t2 == MRS_GEOM_BOX) {
#ifdef MRS_DIAG_NOBB
    return 0;  // diagnostic build only: no box-box contacts
#endif
    int n;
#ifdef MRS_BB_INLINE
    if constexpr (G == 64) {
      [[clang::always_inline]] n = box_box<G>(gxpos, gxmat, gsize, g1, g2, margin, out);
    } else
#endif
    {
      [[clang::noinline]] n = box_box<G>(gxpos, gxmat, gsize, g1, g2, margin, out);
    }
    return n;
  }
  // every other pair has an ellipsoid, cylinder or mesh: general convex (MPR)
  return convex_convex(m, g1, g2, p1, m1, s1, p2, m2, s2, margin, out);
}
// mju_makeFrame: tangent basis from the contact normal
__device__ __forceinline__ void make_frame(float f[9]) {
  normalize3(f);
  if (fabsf(f[1]) < 0.5f) { f[3] = 0; f[4] = 1; f[5] = 0; }
  else { f[3] = 0; f[4] = 0; f[5] = 1; }
  float dd = dot3(f, f + 3);
  for (int i = 0; i < 3; ++i) f[3 + i] -= dd * f[i];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}

template <class PS>
__device__ __forceinline__ float impedance(const PS si, float pos, float margin) {
  float dmin = clampf(si[0], 0.0001f, 0.9999f), dmax = clampf(si[1], 0.0001f, 0.9999f);
  float width = si[2], mid = si[3], power = si[4];
  if (dmin == dmax || width <= kMinVal) return 0.5f * (dmin + dmax);
  float x = fabsf(pos - margin) / width;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  float y;
  if (power == 1) y = x;
  else if (x <= mid) y = powf(x, power) / powf(mid, power - 1);
  else y = 1 - powf(1 - x, power) / powf(1 - mid, power - 1);
  return dmin + y * (dmax - dmin);
}

enum { EFC_FRICTION = 1, EFC_LIMIT = 2, EFC_CONTACT = 3, EFC_EQUALITY = 4, EFC_TFRICTION = 5, EFC_TLIMIT = 6 };
// equality rows are unbounded: the solvers treat them as friction-loss rows with this bound (oracle.c
// EQ_BOUND), quadratic in every primal state and unclamped in PGS
constexpr float kEqBound = 1e15f;
__device__ __forceinline__ bool fric_like(int t) { return t == EFC_FRICTION || t == EFC_EQUALITY || t == EFC_TFRICTION; }

// Per-phase cycle accounting, built only with -DMRS_PHASE_TIMING (profiling variant): s_memtime
// around each phase, summed per wave and added to a device table at the end of the kernel.
enum { PH_KIN, PH_COMPOS, PH_MAKEM, PH_CHOL, PH_COMVEL, PH_RNE, PH_SMOOTH, PH_COLL, PH_CONSTR, PH_SENS,
       PH_INTEG, PH_CHECK, PH_SENS_L1, PH_SENS_SETUP, PH_SENS_GEOMS, PH_CON_ROWS, PH_CON_REC, PH_CON_WARM,
       PH_CON_PGS, PH_COLL_NARROW, PH_COLL_OUT, PH_CON_DEL, PH_REC_J, PH_REC_SOLVE, PH_REC_ROWS, PH_COUNT };
#ifdef MRS_PHASE_TIMING
__device__ unsigned long long g_phase_cycles[PH_COUNT];
#define SUB_T() __builtin_amdgcn_s_memtime()
#define SUB_ADD(id, t0)                                                              \
  do {                                                                               \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();                     \
    if (__lane_id() == 0) atomicAdd(&g_phase_cycles[id], t1_ - (t0));                \
  } while (0)
#else
#define SUB_T() 0ull
#define SUB_ADD(id, t0) (void)(t0)
#endif
#ifdef MRS_PHASE_TIMING
#define PH_BEGIN() unsigned long long ph_t0_ = __builtin_amdgcn_s_memtime()
#define PH_END(acc, id)                                         \
  do {                                                          \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
    (acc)[id] += t1_ - ph_t0_;                                  \
    ph_t0_ = t1_;                                               \
  } while (0)
#define PH_ACC_PARAM , unsigned long long* ph_acc
#define PH_ACC_ARG , ph_acc
#else
#define PH_BEGIN() (void)0
#define PH_END(acc, id) (void)0
#define PH_ACC_PARAM
#define PH_ACC_ARG
#endif

// ------------------------------------------------------------------ environment context
// Phases are separate non-inlined functions (own register allocation, nothing live across them
// but these four values).  The model (with its LDS/scratch layouts) stays in device memory behind
// one pointer: wave-uniform model reads become scalar loads instead of SGPR-resident kernel args.
#define ENV_PARAMS const DevModel* __restrict__ mp, lfloat* __restrict__ s, gfloat* __restrict__ scr, int lane
#define ENV_ARGS mp, s, scr, lane
// Function arguments arrive in VGPRs, so the compiler cannot know they are wave-uniform; the phase
// prologue re-establishes uniformity with readfirstlane (every phase is entered by the whole wave).
// With several environments per wave (G < 64) only the model pointer is wave-uniform; the LDS base
// and scratch pointers of each group stay per-lane.
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v));
  const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v >> 32));
  return reinterpret_cast<T*>((static_cast<unsigned long long>(hi) << 32) | lo);
}
__device__ __forceinline__ lfloat* uniform_lds(lfloat* p) {
  return (lfloat*)(unsigned long)__builtin_amdgcn_readfirstlane((unsigned)(unsigned long)p);
}
__device__ __forceinline__ int uniform_int(int v) { return __builtin_amdgcn_readfirstlane(v); }

// the workgroup-shared LDS tables (DevModel::shr_*), staged by step_kernel at launch
extern __shared__ __attribute__((aligned(16))) float g_dyn_lds[];
__device__ __forceinline__ const lfloat* shared_lds(const DevModel& m) { return (const lfloat*)(g_dyn_lds + m.shr_off); }
// helper waves' one-way signal (step_kernel): each physics wave counts its com_pos passes in a
// workgroup LDS word of its own (release: com_pos's LDS writes land first); its helper wave waits for
// the count it needs (acquire) before building the rows from them, so the physics wave never waits for
// the helper there.  One word per physics wave (DevModel::shr_flag, 4 words), so the protocol holds
// for any number of physics waves per workgroup.  The wait gives up after ~2^26 polls (seconds), far
// past any real step, so that a broken protocol cannot hang the device; it then returns false, the
// helper leaves the rows to the physics wave (which builds them inline from its own com_pos) and
// counts the timeout in the env's warning[3] (MRS_FIELD_WARNING) -- never silently stale rows.
__device__ __forceinline__ int* helper_flag(const DevModel& m, int wave) {
  return (int*)(g_dyn_lds + m.shr_off + m.shr_flag) + wave;
}
__device__ __forceinline__ void helper_signal(const DevModel& m, int wave) {
  if (__lane_id() == 0) __hip_atomic_fetch_add(helper_flag(m, wave), 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool helper_wait(const DevModel& m, int wave, int count) {
  for (unsigned k = 0; k < (1u << 26); ++k) {
    if (__hip_atomic_load(helper_flag(m, wave), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= count) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}
// by-value copy of the model descriptor read through the constant address space: only the fields a
// phase uses are loaded (scalar loads), and they stay in SGPRs for the whole phase
__device__ __forceinline__ DevModel load_model(const DevModel* mp) {
  DevModel m;
  __builtin_memcpy(&m, (const __attribute__((address_space(4))) DevModel*)mp, sizeof(DevModel));
  return m;
}

#define ENV_UNPACK                        \
  mp = uniform_ptr(mp);                   \
  if constexpr (G == 64) {                \
    s = uniform_lds(s);                   \
    scr = uniform_ptr(scr);               \
  }                                       \
  lane = __lane_id() & (G - 1);           \
  const DevModel m = load_model(mp); \
  const LdsLayout& L = m.L;         \
  const ScratchLayout& S = m.S;     \
  (void)L; (void)S; (void)scr; (void)lane

// Index of M(i, j) (i, j in one kinematic tree) in the LDS storage of M and its factor: dense
// nv x nv rows, or (blocked mode, one env per wave) the row-major block of the dofs' tree.
template <int G>
__device__ __forceinline__ int midx(const DevModel& m, int i, int j) {
  if constexpr (G == 64) {
    const int t = m.dof_tree[i], a = m.tree_dofadr[t], n = m.tree_dofnum[t];
    return m.tree_Moff[t] + (i - a) * n + (j - a);
  } else {
    return i * m.nv + j;
  }
}

// Cholesky of the dense nv x nv matrix A (LDS) into Lf (LDS), column by column; lanes over rows.
// Blocked mode (G = 64): every tree's block at once, columns up to the largest tree's size.
// G = 16 dense factor, N = unroll bound >= nv: lane i keeps row i of A and then of L in registers;
// column k needs L[k][p] for p < k, which is lane k's register p: one DPP row broadcast each, no LDS
// round trip in the chain
template <int N>
__device__ __forceinline__ void chol_rows16(const lfloat* A, lfloat* Lf, int nv, int lane) {
  float row[N];
  unroll<N>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    row[p] = (p < nv && lane < nv) ? A[lane * nv + p] : 0.0f;
  });
  unroll<N>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if (k < nv) {
      float t = row[k];
      unroll<k>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        t -= row[p] * rowb<k>(row[p]);
      });
      const float dk = rowb<k>(t);
      const float lkk = sqrtf(dk > kMinVal ? dk : kMinVal);
      row[k] = lane == k ? lkk : (lane > k ? t / lkk : row[k]);
    }
  });
  if (lane < nv)
    unroll<N>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      if (p < nv) Lf[lane * nv + p] = p <= lane ? row[p] : 0.0f;
    });
}

// two factors in one pass: M (into Lf) and M + diag(h dg) (into Lh, which may alias A): the same
// register row form, the two column chains interleaved so each hides the other's latency
// (DevModel::fuse_ih); the diagonal update is integrate()'s fma, so both factors are bit-identical to
// the separate ones
template <int N>
__device__ __forceinline__ void chol_rows16_dual(const lfloat* A, lfloat* Lf, lfloat* Lh, float h, float dg, int nv,
                                                 int lane) {
  float ra[N], rb[N];
  unroll<N>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    ra[p] = (p < nv && lane < nv) ? A[lane * nv + p] : 0.0f;
    rb[p] = p == lane ? __builtin_fmaf(h, dg, ra[p]) : ra[p];
  });
  unroll<N>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if (k < nv) {
      float ta = ra[k], tb = rb[k];
      unroll<k>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        ta -= ra[p] * rowb<k>(ra[p]);
        tb -= rb[p] * rowb<k>(rb[p]);
      });
      const float da = rowb<k>(ta), db = rowb<k>(tb);
      const float la = sqrtf(da > kMinVal ? da : kMinVal), lb = sqrtf(db > kMinVal ? db : kMinVal);
      ra[k] = lane == k ? la : (lane > k ? ta / la : ra[k]);
      rb[k] = lane == k ? lb : (lane > k ? tb / lb : rb[k]);
    }
  });
  wsync();  // (Lh may alias A: every lane has read its row)
  if (lane < nv)
    unroll<N>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      if (p < nv) {
        Lf[lane * nv + p] = p <= lane ? ra[p] : 0.0f;
        Lh[lane * nv + p] = p <= lane ? rb[p] : 0.0f;
      }
    });
}

template <int G>
__device__ MRS_PHASE void cholesky(const DevModel* __restrict__ mp, const lfloat* A, lfloat* Lf, int lane) {
  mp = uniform_ptr(mp);
  if constexpr (G == 64) {
    A = uniform_lds(const_cast<lfloat*>(A));
    Lf = uniform_lds(Lf);
  }
  lane = __lane_id() & (G - 1);
  const int nv = load_model(mp).nv;
  if constexpr (G == 16) {
    // unrolled to 8 dofs when nv <= 8 (a quarter of the code of the 16-dof form)
    if (nv <= 8) chol_rows16<8>(A, Lf, nv, lane);
    else chol_rows16<16>(A, Lf, nv, lane);
    wsync();
    return;
  }
  if constexpr (G == 64) {
    const DevModel m = load_model(mp);
    const int tr = lane < nv ? m.dof_tree[lane] : 0;
    const int a = m.tree_dofadr[tr], n = lane < nv ? m.tree_dofnum[tr] : 0, li = lane - a;
    const lfloat* Ab = A + m.tree_Moff[tr];
    lfloat* Lb = Lf + m.tree_Moff[tr];
    #pragma unroll 1
    for (int k = 0; k < m.tree_nmax; ++k) {
      float t = 0;
      if (li >= k && k < n) {
        t = Ab[li * n + k];
        for (int p = 0; p < k; ++p) t -= Lb[li * n + p] * Lb[k * n + p];
      }
      const float dk = __shfl(t, a + k);  // pivot lane of this lane's tree (unused when k >= n)
      const float lkk = sqrtf(dk > kMinVal ? dk : kMinVal);
      if (k < n) {
        if (li == k) Lb[k * n + k] = lkk;
        else if (li > k) Lb[li * n + k] = t / lkk;
      }
      wsync();
    }
    return;
  }
  #pragma unroll 1
  for (int k = 0; k < nv; ++k) {
    float t = 0;
    if (lane >= k && lane < nv) {
      t = A[lane * nv + k];
      for (int p = 0; p < k; ++p) t -= Lf[lane * nv + p] * Lf[k * nv + p];
    }
    float dk = gbcast<G>(t, k);
    float lkk = sqrtf(dk > kMinVal ? dk : kMinVal);
    if (lane == k) Lf[k * nv + k] = lkk;
    else if (lane > k && lane < nv) Lf[lane * nv + k] = t / lkk;
    wsync();
  }
}
// x = A^-1 b with A = Lf Lf'; lane j holds b_j / returns x_j (lanes >= nv return 0)
// G = 16 solve, N = unroll bound >= nv: lane j prefetches row j of L (forward) and column j
// (backward); the substitution chains are DPP broadcasts and FMAs
template <int N>
__device__ __forceinline__ float chol_solve_rows16(const lfloat* Lf, float x, int nv, int lane) {
  float lrow[N], lcol[N], inv[N];
  unroll<N>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    lrow[i] = (i < nv && lane < nv) ? Lf[lane * nv + i] : 0.0f;
    lcol[i] = (i < nv && lane < nv) ? Lf[i * nv + lane] : 0.0f;
    inv[i] = i < nv ? 1.0f / Lf[i * nv + i] : 0.0f;
  });
  unroll<N>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if (i < nv) {
      const float xi = rowb<i>(x) * inv[i];
      x = lane == i ? xi : (lane > i ? x - lrow[i] * xi : x);
    }
  });
  unroll<N>([&](auto ic) {
    constexpr int i = N - 1 - decltype(ic)::value;
    if (i < nv) {
      const float xi = rowb<i>(x) * inv[i];
      x = lane == i ? xi : (lane < i ? x - lcol[i] * xi : x);
    }
  });
  return x;
}

template <int G>
__device__ MRS_PHASE float chol_solve_lanes(const DevModel* __restrict__ mp, const lfloat* Lf, float b, int lane) {
  mp = uniform_ptr(mp);
  if constexpr (G == 64) Lf = uniform_lds(const_cast<lfloat*>(Lf));
  lane = __lane_id() & (G - 1);
  const int nv = load_model(mp).nv;
  float x = lane < nv ? b : 0.0f;
  if constexpr (G == 16) {
    x = nv <= 8 ? chol_solve_rows16<8>(Lf, x, nv, lane) : chol_solve_rows16<16>(Lf, x, nv, lane);
    return lane < nv ? x : 0.0f;
  }
  if constexpr (G == 64) {
    // per tree block: lane of local index k is the pivot of step k
    const DevModel m = load_model(mp);
    const int tr = lane < nv ? m.dof_tree[lane] : 0;
    const int a = m.tree_dofadr[tr], n = lane < nv ? m.tree_dofnum[tr] : 0, li = lane - a;
    const lfloat* Lb = Lf + m.tree_Moff[tr];
    #pragma unroll 1
    for (int k = 0; k < m.tree_nmax; ++k) {
      const float xs = __shfl(x, a + k);
      if (k < n) {
        const float xk = xs / Lb[k * n + k];
        if (li == k) x = xk;
        else if (li > k) x -= Lb[li * n + k] * xk;
      }
    }
    #pragma unroll 1
    for (int k = m.tree_nmax - 1; k >= 0; --k) {
      const float xs = __shfl(x, a + k);
      if (k < n) {
        const float xk = xs / Lb[k * n + k];
        if (li == k) x = xk;
        else if (li < k) x -= Lb[k * n + li] * xk;
      }
    }
    return lane < nv ? x : 0.0f;
  }
  #pragma unroll 1
  for (int i = 0; i < nv; ++i) {
    float xi = gbcast<G>(x, i) / Lf[i * nv + i];
    if (lane == i) x = xi;
    else if (lane > i && lane < nv) x -= Lf[lane * nv + i] * xi;
  }
  for (int i = nv - 1; i >= 0; --i) {
    float xi = gbcast<G>(x, i) / Lf[i * nv + i];
    if (lane == i) x = xi;
    else if (lane < i) x -= Lf[i * nv + lane] * xi;
  }
  return x;
}
// serial solve by one lane (vectors in registers/scratch); used per constraint row
__device__ __forceinline__ void chol_solve_serial(const lfloat* Lf, int nv, const gfloat* b, gfloat* x) {
  #pragma unroll 1
  for (int i = 0; i < nv; ++i) {
    float sacc = b[i];
    for (int k = 0; k < i; ++k) sacc -= Lf[i * nv + k] * x[k];
    x[i] = sacc / Lf[i * nv + i];
  }
  for (int i = nv - 1; i >= 0; --i) {
    float sacc = x[i];
    #pragma unroll 1
    for (int k = i + 1; k < nv; ++k) sacc -= Lf[k * nv + i] * x[k];
    x[i] = sacc / Lf[i * nv + i];
  }
}

// Smooth-dynamics tables (batch.hip actrec, dofrec, bodytab, mpairtab): from workgroup LDS with lane
// groups, from the model block in blocked mode (G = 64, where LDS is per env)
template <int G>
__device__ __forceinline__ auto act_tab(const DevModel& m, int a) {
  if constexpr (G == 64) return m.actrec + 20 * a; else return shared_lds(m) + m.shr_act + 20 * a;
}
template <int G>
__device__ __forceinline__ auto dof_tab(const DevModel& m, int j) {
  if constexpr (G == 64) return m.dofrec + 16 * j; else return shared_lds(m) + m.shr_dof + 16 * j;
}
// per body: mass, subtree mass, root, parent, subtree end, dof address, dof count
template <int G>
__device__ __forceinline__ auto body_tab(const DevModel& m, int b) {
  if constexpr (G == 64) return m.bodytab + 8 * b; else return shared_lds(m) + m.shr_body + 8 * b;
}
template <int G>
__device__ __forceinline__ auto mpair_tab(const DevModel& m, int p) {
  if constexpr (G == 64) return m.mpairtab + 4 * p; else return shared_lds(m) + m.shr_mpair + 4 * p;
}
// kinematics tables (batch.hip kinbody / kinjnt / kingeom): from workgroup LDS with lane groups -- the
// per-lane model reads of the kinematics were global loads, which wait (vmcnt counts stores too) for
// the previous step's sensordata stores -- from the model block in blocked mode
template <int G>
__device__ __forceinline__ auto kin_body(const DevModel& m, int b) {
  if constexpr (G == 64) return m.kinbody + 25 * b; else return shared_lds(m) + m.shr_kbody + 25 * b;
}
template <int G>
__device__ __forceinline__ auto kin_jnt(const DevModel& m, int j) {
  if constexpr (G == 64) return m.kinjnt + 13 * j; else return shared_lds(m) + m.shr_kjnt + 13 * j;
}
template <int G>
__device__ __forceinline__ auto kin_geom(const DevModel& m, int g) {
  if constexpr (G == 64) return m.kingeom + 9 * g; else return shared_lds(m) + m.shr_kgeom + 9 * g;
}

// pose of body b from its parent's frame (P, Q): body offset, then its joints in order (mj_kinematics
// per body).  With kJoints the world anchors/axes of the joints are written (P, Q must be the
// parent's world frame then).  A free joint gives the world pose directly (its parent is the world).
template <int G, bool kJoints>
__device__ __forceinline__ void body_pose(const DevModel& m, lfloat* s, int b, const float P[3], const float Q[4],
                                          float pos[3], float q[4]) {
  const LdsLayout& L = m.L;
  const auto kb = kin_body<G>(m, b);
  const int ja = __float_as_int(kb[17]), nj = __float_as_int(kb[18]);
  if (nj > 0 && __float_as_int(kin_jnt<G>(m, ja)[7]) == MRS_JNT_FREE) {
    const lfloat* qp = s + L.qpos + __float_as_int(kin_jnt<G>(m, ja)[6]);
    pos[0] = qp[0]; pos[1] = qp[1]; pos[2] = qp[2];
    q[0] = qp[3]; q[1] = qp[4]; q[2] = qp[5]; q[3] = qp[6];
    quat_normalize(q);
    if (kJoints) {
      lfloat* anc = s + L.xanchor + 3 * ja;
      lfloat* ax = s + L.xaxis + 3 * ja;
      for (int i = 0; i < 3; ++i) { anc[i] = pos[i]; ax[i] = 0; }
    }
    return;
  }
  const float bpos[3] = {kb[0], kb[1], kb[2]};
  const float bq[4] = {kb[3], kb[4], kb[5], kb[6]};
  float r[3];
  rot_quat(r, bpos, Q);
  for (int i = 0; i < 3; ++i) pos[i] = P[i] + r[i];
  quat_mul(q, Q, bq);
  #pragma unroll 1
  for (int k2 = 0; k2 < nj; ++k2) {
    const int j = ja + k2;
    const auto kj = kin_jnt<G>(m, j);
    const int qa = __float_as_int(kj[6]);
    const float jp[3] = {kj[0], kj[1], kj[2]};
    const float ja3[3] = {kj[3], kj[4], kj[5]};
    float anc[3], ax[3];
    rot_quat(anc, jp, q);
    for (int i = 0; i < 3; ++i) anc[i] += pos[i];
    rot_quat(ax, ja3, q);
    if (kJoints)
      for (int i = 0; i < 3; ++i) { s[L.xanchor + 3 * j + i] = anc[i]; s[L.xaxis + 3 * j + i] = ax[i]; }
    const int jt = __float_as_int(kj[7]);
    if (jt == MRS_JNT_SLIDE) {
      const float dq = s[L.qpos + qa] - kj[8];
      for (int i = 0; i < 3; ++i) pos[i] += ax[i] * dq;
    } else {
      float ql[4];
      if (jt == MRS_JNT_BALL) {
        for (int i = 0; i < 4; ++i) ql[i] = s[L.qpos + qa + i];
        quat_normalize(ql);
      } else {
        axis_angle_quat(ql, ja3, s[L.qpos + qa] - kj[8]);
      }
      quat_mul(q, q, ql);
      float v[3];
      rot_quat(v, jp, q);
      for (int i = 0; i < 3; ++i) pos[i] = anc[i] - v[i];
    }
  }
}

// body frame outputs: xpos, xquat, xmat, inertial frame and the rotational part of cinert
template <int G>
__device__ __forceinline__ void body_frame_out(const DevModel& m, lfloat* s, int b, const float pos[3], float q[4]) {
  const LdsLayout& L = m.L;
  const auto kb = kin_body<G>(m, b);
  quat_normalize(q);
  float xm[9];
  quat2mat(xm, q);
  for (int i = 0; i < 3; ++i) s[L.xpos + 3 * b + i] = pos[i];
  for (int i = 0; i < 4; ++i) s[L.xquat + 4 * b + i] = q[i];
  for (int i = 0; i < 9; ++i) s[L.xmat + 9 * b + i] = xm[i];
  // inertial frame; world-frame rotational inertia about the body com goes to cinert[0..5]
  const float ip[3] = {kb[7], kb[8], kb[9]};
  const float iq[4] = {kb[10], kb[11], kb[12], kb[13]};
  float r[3], qi[4], R[9];
  mat_vec(r, xm, ip);
  for (int i = 0; i < 3; ++i) s[L.xipos + 3 * b + i] = pos[i] + r[i];
  quat_mul(qi, q, iq);
  quat2mat(R, qi);
  const float I0 = kb[14], I1 = kb[15], I2 = kb[16];
  lfloat* ci = s + L.cinert + 10 * b;
  ci[0] = R[0] * I0 * R[0] + R[1] * I1 * R[1] + R[2] * I2 * R[2];
  ci[1] = R[3] * I0 * R[3] + R[4] * I1 * R[4] + R[5] * I2 * R[5];
  ci[2] = R[6] * I0 * R[6] + R[7] * I1 * R[7] + R[8] * I2 * R[8];
  ci[3] = R[0] * I0 * R[3] + R[1] * I1 * R[4] + R[2] * I2 * R[5];
  ci[4] = R[0] * I0 * R[6] + R[1] * I1 * R[7] + R[2] * I2 * R[8];
  ci[5] = R[3] * I0 * R[6] + R[4] * I1 * R[7] + R[5] * I2 * R[8];
}

// mj_kinematics + rotational part of cinert.  With one lane per body (nbody <= G) the tree is
// composed by pointer jumping: every body's pose relative to its parent in parallel, then
// ceil(log2(max_depth)) rounds T(b) <- T(ancestor at 2^r) o T(b), then every body again from its
// parent's world pose (joint anchors/axes, frames, inertia).  Otherwise bodies of one depth level
// per pass.
// kinematics of trees with more bodies than the group has lanes: level by level from the root
template <int G>
__device__ void kinematics_levels(ENV_PARAMS) {
  ENV_UNPACK;
  const float P0[3] = {0, 0, 0};
    if (lane == 0) {
      float q1[4] = {1, 0, 0, 0};
      body_frame_out<G>(m, s, 0, P0, q1);
    }
    wsync();
    for (int lev = 1; lev <= m.max_depth; ++lev) {
      const int a0 = m.level_adr[lev], nl = m.level_num[lev];
      #pragma unroll 1
      for (int k = lane; k < nl; k += G) {
        const int b = m.level_body[a0 + k];
        const int p = m.body_parentid[b];
        const float P[3] = {s[L.xpos + 3 * p], s[L.xpos + 3 * p + 1], s[L.xpos + 3 * p + 2]};
        const float Q[4] = {s[L.xquat + 4 * p], s[L.xquat + 4 * p + 1], s[L.xquat + 4 * p + 2], s[L.xquat + 4 * p + 3]};
        float pos[3], q[4];
        body_pose<G, true>(m, s, b, P, Q, pos, q);
        body_frame_out<G>(m, s, b, pos, q);
      }
      wsync();
    }
}

template <int G>
__device__ MRS_PHASE void kinematics(ENV_PARAMS) {
  ENV_UNPACK;
  const float P0[3] = {0, 0, 0}, Q0[4] = {1, 0, 0, 0};
  if (m.nbody <= G) {
    const int b = lane;
    float pos[3] = {0, 0, 0}, q[4] = {1, 0, 0, 0};
    if (b >= 1 && b < m.nbody) body_pose<G, false>(m, s, b, P0, Q0, pos, q);
    if (b < m.nbody) {
      for (int i = 0; i < 3; ++i) s[L.xpos + 3 * b + i] = pos[i];
      for (int i = 0; i < 4; ++i) s[L.xquat + 4 * b + i] = q[i];
    }
    wsync();
    #pragma unroll 1
    for (int r = 0; r < m.njump; ++r) {
      int a = -1;
      if (b >= 1 && b < m.nbody) {
        if constexpr (G == 64) a = m.jump[r * m.nbody + b];
        else a = __float_as_int(shared_lds(m)[m.shr_jump + r * m.nbody + b]);
      }
      float ap[3], aq[4];
      if (a >= 0) {
        for (int i = 0; i < 3; ++i) ap[i] = s[L.xpos + 3 * a + i];
        for (int i = 0; i < 4; ++i) aq[i] = s[L.xquat + 4 * a + i];
      }
      wsync();
      if (a >= 0) {
        float rr[3];
        rot_quat(rr, pos, aq);
        for (int i = 0; i < 3; ++i) pos[i] = ap[i] + rr[i];
        quat_mul(q, aq, q);
        for (int i = 0; i < 3; ++i) s[L.xpos + 3 * b + i] = pos[i];
        for (int i = 0; i < 4; ++i) s[L.xquat + 4 * b + i] = q[i];
      }
      wsync();
    }
    if (m.kin_onepass) {
      // (every body has no joint or one hinge / free joint) the jumps left each body's world pose in
      // pos / q, and its joint frame follows from that pose: a hinge turns the body about the joint's
      // anchor and axis, so both are the same before and after the rotation -- xanchor = xpos + R jnt_pos,
      // xaxis = R jnt_axis (mj_kinematics computes them before applying the joint); a free joint's
      // anchor is the body position, axis 0.  No second pass from the parents' poses.
      if (b >= 1 && b < m.nbody) {
        quat_normalize(q);
        const auto kb = kin_body<G>(m, b);
        if (__float_as_int(kb[18]) == 1) {
          const int j = __float_as_int(kb[17]);
          const auto kj = kin_jnt<G>(m, j);
          float anc[3] = {pos[0], pos[1], pos[2]}, ax[3] = {0, 0, 0};
          if (__float_as_int(kj[7]) == MRS_JNT_HINGE) {
            const float jp[3] = {kj[0], kj[1], kj[2]}, ja3[3] = {kj[3], kj[4], kj[5]};
            float r[3];
            rot_quat(r, jp, q);
            for (int i = 0; i < 3; ++i) anc[i] += r[i];
            rot_quat(ax, ja3, q);
          }
          for (int i = 0; i < 3; ++i) { s[L.xanchor + 3 * j + i] = anc[i]; s[L.xaxis + 3 * j + i] = ax[i]; }
        }
        body_frame_out<G>(m, s, b, pos, q);
      } else if (b == 0) {
        float q1[4] = {1, 0, 0, 0};
        body_frame_out<G>(m, s, 0, P0, q1);
      }
      wsync();
    } else {
    // every body from its parent's world pose (same values up to rounding, plus joint frames)
    float P[3] = {0, 0, 0}, Q[4] = {1, 0, 0, 0};
    if (b >= 1 && b < m.nbody) {
      const int p = __float_as_int(body_tab<G>(m, b)[3]);
      for (int i = 0; i < 3; ++i) P[i] = s[L.xpos + 3 * p + i];
      for (int i = 0; i < 4; ++i) Q[i] = s[L.xquat + 4 * p + i];
    }
    wsync();
    if (b >= 1 && b < m.nbody) {
      body_pose<G, true>(m, s, b, P, Q, pos, q);
      body_frame_out<G>(m, s, b, pos, q);
    } else if (b == 0) {
      float q1[4] = {1, 0, 0, 0};
      body_frame_out<G>(m, s, 0, P0, q1);
    }
    wsync();
    }
  } else {
    MRS_COLD(G, kinematics_levels<G>(ENV_ARGS));
  }
  // geoms
  #pragma unroll 1
  for (int g = lane; g < m.ngeom; g += G) {
    const auto kg = kin_geom<G>(m, g);
    const int b = __float_as_int(kg[0]);
    float bq[4] = {s[L.xquat + 4 * b], s[L.xquat + 4 * b + 1], s[L.xquat + 4 * b + 2], s[L.xquat + 4 * b + 3]};
    float gp[3] = {kg[1], kg[2], kg[3]};
    float gq[4] = {kg[4], kg[5], kg[6], kg[7]};
    float r[3], q[4], gm[9];
    rot_quat(r, gp, bq);
    for (int i = 0; i < 3; ++i) s[L.gxpos + 3 * g + i] = s[L.xpos + 3 * b + i] + r[i];
    quat_mul(q, bq, gq);
    quat2mat(gm, q);
    for (int i = 0; i < 9; ++i) s[L.gxmat + 9 * g + i] = gm[i];
  }
  wsync();
}

// mj_comPos: subtree coms of tree roots, cinert (parallel-axis part), cdof
template <int G>
__device__ MRS_PHASE void com_pos(ENV_PARAMS) {
  ENV_UNPACK;
  #pragma unroll 1
  for (int b = lane; b < m.nbody; b += G) {
    const auto bt = body_tab<G>(m, b);
    if (b != 0 && __float_as_int(bt[3]) != 0) continue;
    float c[3] = {0, 0, 0};
    const int e = __float_as_int(bt[4]);
    #pragma unroll 4
    for (int k = b; k < e; ++k) {
      const float mk = body_tab<G>(m, k)[0];
      for (int i = 0; i < 3; ++i) c[i] += mk * s[L.xipos + 3 * k + i];
    }
    const float sm = bt[1];
    for (int i = 0; i < 3; ++i) s[L.scom + 3 * b + i] = sm > kMinVal ? c[i] / sm : s[L.xipos + 3 * b + i];
  }
  wsync();
  #pragma unroll 1
  for (int b = lane; b < m.nbody; b += G) {
    lfloat* ci = s + L.cinert + 10 * b;
    if (b == 0) { for (int i = 0; i < 10; ++i) ci[i] = 0; continue; }
    const auto bt = body_tab<G>(m, b);
    const int rt = __float_as_int(bt[2]);
    const float mass = bt[0];
    float d[3];
    for (int i = 0; i < 3; ++i) d[i] = s[L.xipos + 3 * b + i] - s[L.scom + 3 * rt + i];
    ci[0] += mass * (d[1] * d[1] + d[2] * d[2]);
    ci[1] += mass * (d[0] * d[0] + d[2] * d[2]);
    ci[2] += mass * (d[0] * d[0] + d[1] * d[1]);
    ci[3] -= mass * d[0] * d[1];
    ci[4] -= mass * d[0] * d[2];
    ci[5] -= mass * d[1] * d[2];
    ci[6] = mass * d[0]; ci[7] = mass * d[1]; ci[8] = mass * d[2]; ci[9] = mass;
  }
  #pragma unroll 1
  for (int j = lane; j < m.njnt; j += G) {
    const auto kj = kin_jnt<G>(m, j);
    const int b = __float_as_int(kj[9]), rt = __float_as_int(kj[11]);
    int dof = __float_as_int(kj[10]);
    float off[3];
    for (int i = 0; i < 3; ++i) off[i] = s[L.scom + 3 * rt + i] - s[L.xanchor + 3 * j + i];
    const int jt = __float_as_int(kj[7]);
    if (jt == MRS_JNT_HINGE) {
      lfloat* cd = s + L.cdof + 6 * dof;
      float ax[3] = {s[L.xaxis + 3 * j], s[L.xaxis + 3 * j + 1], s[L.xaxis + 3 * j + 2]}, c[3];
      cross3(c, ax, off);
      for (int i = 0; i < 3; ++i) { cd[i] = ax[i]; cd[3 + i] = c[i]; }
    } else if (jt == MRS_JNT_SLIDE) {
      lfloat* cd = s + L.cdof + 6 * dof;
      for (int i = 0; i < 3; ++i) { cd[i] = 0; cd[3 + i] = s[L.xaxis + 3 * j + i]; }
    } else {
      if (jt == MRS_JNT_FREE) {
        for (int k = 0; k < 3; ++k)
          for (int i = 0; i < 6; ++i) s[L.cdof + 6 * (dof + k) + i] = (i == 3 + k) ? 1.0f : 0.0f;
        dof += 3;
      }
      for (int k = 0; k < 3; ++k) {
        float ax[3] = {s[L.xmat + 9 * b + k], s[L.xmat + 9 * b + 3 + k], s[L.xmat + 9 * b + 6 + k]}, c[3];
        cross3(c, ax, off);
        lfloat* cd = s + L.cdof + 6 * (dof + k);
        for (int i = 0; i < 3; ++i) { cd[i] = ax[i]; cd[3 + i] = c[i]; }
      }
    }
  }
  wsync();
}

// mj_crb + armature: crb by subtree sums, M by (dof, ancestor-dof) pairs
template <int G>
__device__ MRS_PHASE void make_M(ENV_PARAMS) {
  ENV_UNPACK;
  const int nv = m.nv;
  #pragma unroll 1
  for (int b = lane; b < m.nbody; b += G) {
    float acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (b != 0) {
      const int e = __float_as_int(body_tab<G>(m, b)[4]);
      #pragma unroll 4
      for (int k = b; k < e; ++k)
        for (int i = 0; i < 10; ++i) acc[i] += s[L.cinert + 10 * k + i];
    }
    for (int i = 0; i < 10; ++i) s[L.crb + 10 * b + i] = acc[i];
  }
  const int msize = G == 64 ? m.nMblk : nv * nv;
  #pragma unroll 1
  for (int i = lane; i < msize; i += G) s[L.M + i] = 0;
  wsync();
  #pragma unroll 1
  for (int p = lane; p < m.nMpair; p += G) {
    const auto mp4 = mpair_tab<G>(m, p);  // i, j, body of i, armature
    const int i = __float_as_int(mp4[0]), j = __float_as_int(mp4[1]);
    float buf[6], cd[6];
    for (int k = 0; k < 6; ++k) cd[k] = s[L.cdof + 6 * i + k];
    mul_inert_vec(buf, s + L.crb + 10 * __float_as_int(mp4[2]), cd);
    float v = mp4[3];
    for (int k = 0; k < 6; ++k) v += s[L.cdof + 6 * j + k] * buf[k];
    s[L.M + midx<G>(m, i, j)] = v;
    s[L.M + midx<G>(m, j, i)] = v;
  }
  wsync();
}

// prefix sums of a 6-vector down the tree by pointer jumping (one lane per body, nbody <= G):
// on entry lane b holds its own term v, on exit the sum over b and its ancestors (world excluded);
// buf (6 per body) is the exchange buffer and holds the result
template <int G>
__device__ __forceinline__ void tree_prefix6(const DevModel& m, lfloat* buf, int b, float v[6]) {
  if (b < m.nbody)
    for (int i = 0; i < 6; ++i) buf[6 * b + i] = v[i];
  wsync();
  #pragma unroll 1
  for (int r = 0; r < m.njump; ++r) {
    int a = -1;
    if (b >= 1 && b < m.nbody) {
      if constexpr (G == 64) a = m.jump[r * m.nbody + b];
      else a = __float_as_int(shared_lds(m)[m.shr_jump + r * m.nbody + b]);
    }
    float av[6];
    if (a >= 0)
      for (int i = 0; i < 6; ++i) av[i] = buf[6 * a + i];
    wsync();
    if (a >= 0) {
      for (int i = 0; i < 6; ++i) v[i] += av[i];
      for (int i = 0; i < 6; ++i) buf[6 * b + i] = v[i];
    }
    wsync();
  }
}

// cdof_dot of body b's dofs from the velocity of its parent (mj_comVel per body); returns cvel[b]
// (dof and body indices from the tree tables: workgroup LDS with lane groups)
template <int G>
__device__ __forceinline__ void body_comvel(const DevModel& m, lfloat* s, int b, float cv[6]) {
  const LdsLayout& L = m.L;
  const auto bt = body_tab<G>(m, b);
  const int da = __float_as_int(bt[5]), nd = __float_as_int(bt[6]);
  #pragma unroll 1
  for (int k2 = 0; k2 < nd; ++k2) {
    const int j = da + k2;
    const auto dr = dof_tab<G>(m, j);
    const int jt = __float_as_int(dr[5]);
    if (jt == MRS_JNT_FREE && j == __float_as_int(dr[14])) {
      for (int t = 0; t < 3; ++t) {
        const float qv = s[L.qvel + j + t];
        for (int i = 0; i < 6; ++i) {
          s[L.cdofdot + 6 * (j + t) + i] = 0;
          cv[i] += s[L.cdof + 6 * (j + t) + i] * qv;
        }
      }
      k2 += 2;
      continue;
    }
    if (jt == MRS_JNT_BALL || jt == MRS_JNT_FREE) {
      for (int t = 0; t < 3; ++t) cross_motion(s + L.cdofdot + 6 * (j + t), cv, s + L.cdof + 6 * (j + t));
      for (int t = 0; t < 3; ++t) {
        const float qv = s[L.qvel + j + t];
        for (int i = 0; i < 6; ++i) cv[i] += s[L.cdof + 6 * (j + t) + i] * qv;
      }
      k2 += 2;
      continue;
    }
    cross_motion(s + L.cdofdot + 6 * j, cv, s + L.cdof + 6 * j);
    const float qv = s[L.qvel + j];
    for (int i = 0; i < 6; ++i) cv[i] += s[L.cdof + 6 * j + i] * qv;
  }
}

// mj_comVel: pointer jumping (cvel[b] = sum over b and its ancestors of cdof qvel) when nbody <= G,
// then cdof_dot per body from the parent's velocity; level by level otherwise
template <int G>
__device__ void com_vel_levels(ENV_PARAMS);

template <int G>
__device__ MRS_PHASE void com_vel(ENV_PARAMS) {
  ENV_UNPACK;
  if (m.nbody <= G) {
    const int b = lane;
    float v[6] = {0, 0, 0, 0, 0, 0};
    if (b >= 1 && b < m.nbody) {
      const int da = __float_as_int(body_tab<G>(m, b)[5]), nd = __float_as_int(body_tab<G>(m, b)[6]);
      #pragma unroll 1
      for (int j = da; j < da + nd; ++j) {
        const float qv = s[L.qvel + j];
        for (int i = 0; i < 6; ++i) v[i] += s[L.cdof + 6 * j + i] * qv;
      }
    }
    tree_prefix6<G>(m, s + L.cvel, b, v);
    if (b >= 1 && b < m.nbody) {
      const int p = __float_as_int(body_tab<G>(m, b)[3]);
      float cv[6];
      for (int i = 0; i < 6; ++i) cv[i] = s[L.cvel + 6 * p + i];
      body_comvel<G>(m, s, b, cv);
    }
    wsync();
    return;
  }
  MRS_COLD(G, com_vel_levels<G>(ENV_ARGS));
}

// mj_comVel level by level (trees with more bodies than the group has lanes)
template <int G>
__device__ void com_vel_levels(ENV_PARAMS) {
  ENV_UNPACK;
  if (lane < 6) s[L.cvel + lane] = 0;
  wsync();
  for (int lev = 1; lev <= m.max_depth; ++lev) {
    const int a0 = m.level_adr[lev], nl = m.level_num[lev];
    #pragma unroll 1
    for (int k = lane; k < nl; k += G) {
      const int b = m.level_body[a0 + k];
      const int p = m.body_parentid[b];
      float cv[6];
      for (int i = 0; i < 6; ++i) cv[i] = s[L.cvel + 6 * p + i];
      body_comvel<G>(m, s, b, cv);
      for (int i = 0; i < 6; ++i) s[L.cvel + 6 * b + i] = cv[i];
    }
    wsync();
  }
}

// mj_rne (no acceleration term): qfrc_bias.  cacc[b] = -gravity + sum over b and its ancestors of
// cdof_dot qvel (pointer jumping when nbody <= G, else level by level); body forces in parallel;
// subtree sums by DFS ranges
// mj_rne's body accelerations and forces level by level (trees deeper than the group has lanes)
template <int G>
__device__ void rne_levels(ENV_PARAMS) {
  ENV_UNPACK;
  float g0[6] = {0, 0, 0, 0, 0, 0};
  if (!(m.disableflags & MRS_DSBL_GRAVITY)) { g0[3] = -m.gravity[0]; g0[4] = -m.gravity[1]; g0[5] = -m.gravity[2]; }
    if (lane < 6) s[L.cacc + lane] = g0[lane];
    wsync();
    for (int lev = 1; lev <= m.max_depth; ++lev) {
      const int a0 = m.level_adr[lev], nl = m.level_num[lev];
      #pragma unroll 1
      for (int k = lane; k < nl; k += G) {
        const int b = m.level_body[a0 + k];
        float ca[6];
        for (int i = 0; i < 6; ++i) ca[i] = s[L.cacc + 6 * m.body_parentid[b] + i];
        const int da = m.body_dofadr[b], nd = m.body_dofnum[b];
        #pragma unroll 1
        for (int k2 = 0; k2 < nd; ++k2) {
          const float qv = s[L.qvel + da + k2];
          for (int i = 0; i < 6; ++i) ca[i] += s[L.cdofdot + 6 * (da + k2) + i] * qv;
        }
        for (int i = 0; i < 6; ++i) s[L.cacc + 6 * b + i] = ca[i];
        float f1[6], t[6], f2[6], cv[6];
        for (int i = 0; i < 6; ++i) cv[i] = s[L.cvel + 6 * b + i];
        mul_inert_vec(f1, s + L.cinert + 10 * b, ca);
        mul_inert_vec(t, s + L.cinert + 10 * b, cv);
        cross_force(f2, cv, t);
        for (int i = 0; i < 6; ++i) s[L.cfrc + 6 * b + i] = f1[i] + f2[i];
      }
      wsync();
    }
}

template <int G>
__device__ MRS_PHASE void rne(ENV_PARAMS) {
  ENV_UNPACK;
  float g0[6] = {0, 0, 0, 0, 0, 0};
  if (!(m.disableflags & MRS_DSBL_GRAVITY)) { g0[3] = -m.gravity[0]; g0[4] = -m.gravity[1]; g0[5] = -m.gravity[2]; }
  if (m.nbody <= G) {
    const int b = lane;
    float v[6] = {0, 0, 0, 0, 0, 0};
    if (b >= 1 && b < m.nbody) {
      const int da = __float_as_int(body_tab<G>(m, b)[5]), nd = __float_as_int(body_tab<G>(m, b)[6]);
      #pragma unroll 1
      for (int j = da; j < da + nd; ++j) {
        const float qv = s[L.qvel + j];
        for (int i = 0; i < 6; ++i) v[i] += s[L.cdofdot + 6 * j + i] * qv;
      }
    }
    tree_prefix6<G>(m, s + L.cacc, b, v);
    if (b < m.nbody) {
      float ca[6];
      for (int i = 0; i < 6; ++i) ca[i] = v[i] + g0[i];
      for (int i = 0; i < 6; ++i) s[L.cacc + 6 * b + i] = ca[i];
      if (b >= 1) {
        float f1[6], t[6], f2[6], cv[6];
        for (int i = 0; i < 6; ++i) cv[i] = s[L.cvel + 6 * b + i];
        mul_inert_vec(f1, s + L.cinert + 10 * b, ca);
        mul_inert_vec(t, s + L.cinert + 10 * b, cv);
        cross_force(f2, cv, t);
        for (int i = 0; i < 6; ++i) s[L.cfrc + 6 * b + i] = f1[i] + f2[i];
      }
    }
    wsync();
  } else {
    MRS_COLD(G, rne_levels<G>(ENV_ARGS));
  }
  // subtree sums of body forces into crb storage (crb no longer needed)
  #pragma unroll 1
  for (int b = lane; b < m.nbody; b += G) {
    float acc[6] = {0, 0, 0, 0, 0, 0};
    if (b != 0) {
      const int e = __float_as_int(body_tab<G>(m, b)[4]);
      #pragma unroll 4
      for (int k = b; k < e; ++k)
        for (int i = 0; i < 6; ++i) acc[i] += s[L.cfrc + 6 * k + i];
    }
    for (int i = 0; i < 6; ++i) s[L.crb + 6 * b + i] = acc[i];
  }
  wsync();
  #pragma unroll 1
  for (int j = lane; j < m.nv; j += G) {
    const int b = __float_as_int(dof_tab<G>(m, j)[10]);  // body
    float v = 0;
    for (int i = 0; i < 6; ++i) v += s[L.cdof + 6 * j + i] * s[L.crb + 6 * b + i];
    s[L.qfrc_bias + j] = v;
  }
  wsync();
}

// translational point-Jacobian column of dof j for a point on body b (0 if j does not move b)
__device__ __forceinline__ void jac_col(const DevModel& m, const lfloat* s, int b, const float pnt[3], int j, float col[3]) {
  const int bj = m.dof_bodyid[j];
  if (!(b >= bj && b < m.body_subtree_end[bj])) { col[0] = col[1] = col[2] = 0; return; }
  const lfloat* c = s + m.L.scom + 3 * m.body_rootid[b];
  const lfloat* cd = s + m.L.cdof + 6 * j;
  float off[3] = {pnt[0] - c[0], pnt[1] - c[1], pnt[2] - c[2]}, ang[3] = {cd[0], cd[1], cd[2]}, cr[3];
  cross3(cr, ang, off);
  for (int i = 0; i < 3; ++i) col[i] = cd[3 + i] + cr[i];
}

// blocked mode: jac_col with the dof's body and subtree end from the env's LDS table and the body's
// root given (no dependent chain of model-table loads per contact row)
__device__ __forceinline__ void jac_col_blk(const lfloat* s, const LdsLayout& L, int b, int root, const float pnt[3],
                                            int j, float col[3]) {
  const int bj = __float_as_int(s[L.dofb + 2 * j]), be = __float_as_int(s[L.dofb + 2 * j + 1]);
  if (!(b >= bj && b < be)) { col[0] = col[1] = col[2] = 0; return; }
  const lfloat* c = s + L.scom + 3 * root;
  const lfloat* cd = s + L.cdof + 6 * j;
  float off[3] = {pnt[0] - c[0], pnt[1] - c[1], pnt[2] - c[2]}, ang[3] = {cd[0], cd[1], cd[2]}, cr[3];
  cross3(cr, ang, off);
  for (int i = 0; i < 3; ++i) col[i] = cd[3 + i] + cr[i];
}

// mj_passive + mj_fwdActuation + qfrc_smooth + qacc_smooth (lane per dof)
template <int G>
__device__ MRS_PHASE float smooth_forces(ENV_PARAMS) {
  ENV_UNPACK;
  const int nv = m.nv;
  // fixed tendons (mj_tendon): length and velocity of each into the step's tendon slot (lane per tendon)
  if (m.ntendon > 0) {
    #pragma unroll 1
    for (int t = lane; t < m.ntendon; t += G) {
      float len = 0, vel = 0;
      #pragma unroll 1
      for (int k = m.ten_adr[t]; k < m.ten_adr[t] + m.ten_num[t]; ++k) {
        len += m.wrap_coef[k] * s[L.qpos + m.wrap_qadr[k]];
        vel += m.wrap_coef[k] * s[L.qvel + m.wrap_dof[k]];
      }
      s[L.ten + 2 * t] = len;
      s[L.ten + 2 * t + 1] = vel;
    }
    wsync();
  }
  // actuator forces (lane per actuator)
  #pragma unroll 1
  for (int a = lane; a < m.nu; a += G) {
    float force = 0;
    if (!(m.disableflags & MRS_DSBL_ACTUATION)) {
      const auto ar = act_tab<G>(m, a);
      const float gear = ar[2];
      // (a tendon transmission's addresses are -1 - tendon: its length and velocity from the slot)
      const int qad = __float_as_int(ar[0]), dad = __float_as_int(ar[1]);
      const float len = gear * (qad >= 0 ? s[L.qpos + qad] : s[L.ten + 2 * (-1 - qad)]);
      const float vel = gear * (dad >= 0 ? s[L.qvel + dad] : s[L.ten + 2 * (-1 - dad) + 1]);
      float ctrl = s[L.ctrl + a];
      if (__float_as_int(ar[3]) && !(m.disableflags & MRS_DSBL_CLAMPCTRL)) ctrl = clampf(ctrl, ar[4], ar[5]);
      float gain = __float_as_int(ar[6]) == MRS_GAIN_AFFINE ? ar[7] + ar[8] * len + ar[9] * vel : ar[7];
      float bias = __float_as_int(ar[10]) == MRS_BIAS_AFFINE ? ar[11] + ar[12] * len + ar[13] * vel : 0.0f;
      force = gain * ctrl + bias;
      if (__float_as_int(ar[14])) force = clampf(force, ar[15], ar[16]);
    }
    s[L.act_force + a] = force;
  }
  wsync();
  float qfs = 0;
  if (lane < nv) {
    const int j = lane;
    const auto dr = dof_tab<G>(m, j);
    float qa = 0;
    const int da = __float_as_int(dr[0]);
    if (da >= 0) {
      qa = dr[1] * s[L.act_force + da];
    } else if (da == -2) {
      #pragma unroll 1
      for (int a = 0; a < m.nu; ++a) {
        if (m.act_dof[a] == j) qa += m.act_gear[a] * s[L.act_force + a];
        else if (m.ntendon > 0 && m.act_ten[a] >= 0)
          qa += m.act_gear[a] * s[L.act_force + a] * m.ten_J[m.act_ten[a] * nv + j];  // moment gear * J
      }
    }
    if (__float_as_int(dr[2])) qa = clampf(qa, dr[3], dr[4]);
    s[L.qfrc_act + j] = qa;
    float pas = 0;
    if (!(m.disableflags & MRS_DSBL_PASSIVE)) {
      const int jt = __float_as_int(dr[5]);
      if ((jt == MRS_JNT_HINGE || jt == MRS_JNT_SLIDE) && dr[6] != 0) {
        const int qadr = __float_as_int(dr[7]);
        pas -= dr[6] * (s[L.qpos + qadr] - dr[8]);
      }
      pas -= dr[9] * s[L.qvel + j];
      // tendon springs (dead band [lengthspring0, lengthspring1]) and dampers through J'
      #pragma unroll 1
      for (int t = 0; t < m.ntendon; ++t) {
        const float jt = m.ten_J[t * nv + j];
        if (jt == 0) continue;
        const CPtr<float> tp = m.ten_prm + 12 * t;
        const float len = s[L.ten + 2 * t], k = tp[0];
        float f = k == 0 ? 0.0f : (len > tp[3] ? k * (tp[3] - len) : (len < tp[2] ? k * (tp[2] - len) : 0.0f));
        f -= tp[1] * s[L.ten + 2 * t + 1];
        pas += jt * f;
      }
      if (!(m.disableflags & MRS_DSBL_GRAVITY) && __float_as_int(dr[12])) {
        const int bj = __float_as_int(dr[10]), e = __float_as_int(dr[11]);
        #pragma unroll 1
        for (int b = bj; b < e; ++b) {
          const float gc = m.body_gravcomp[b];
          if (gc == 0) continue;
          float f[3], col[3], pnt[3] = {s[L.xipos + 3 * b], s[L.xipos + 3 * b + 1], s[L.xipos + 3 * b + 2]};
          for (int i = 0; i < 3; ++i) f[i] = -m.gravity[i] * m.body_mass[b] * gc;
          jac_col(m, s, b, pnt, j, col);
          pas += dot3(col, f);
        }
      }
    }
    s[L.qfrc_passive + j] = pas;
    qfs = pas - s[L.qfrc_bias + j] + s[L.qfrc_applied + j] + qa;
    s[L.qfrc_smooth + j] = qfs;
  }
  float qacc_s;
  MRS_CALL(G, qacc_s = chol_solve_lanes<G>(mp, s + L.L, qfs, lane));
  if (lane < nv) s[L.qacc_smooth + lane] = qacc_s;
  wsync();
  return qacc_s;
}

__device__ __forceinline__ int wave_max(int v) {
  #pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
// pairs up to which collision() compacts the sphere-test candidates before the narrowphase
constexpr int kCandPairs = 128;

// mj_collision: candidate pairs (lane per pair), bounding-sphere test, narrow phase, compaction
template <int G>
__device__ MRS_PHASE int collision(ENV_PARAMS) {
  ENV_UNPACK;
  int ncon = 0;
  if ((m.disableflags & (MRS_DSBL_CONTACT | MRS_DSBL_CONSTRAINT)) || m.npair == 0) return 0;
  // bounding-sphere test of pair p (planes: always a candidate, mj_collideGeoms)
  auto sphere_cand = [&](int p) {
    const int g1 = m.pair_g1[p], g2 = m.pair_g2[p];
    if (m.geom_type[g1] == MRS_GEOM_PLANE) return true;
    const float dv[3] = {s[L.gxpos + 3 * g1] - s[L.gxpos + 3 * g2], s[L.gxpos + 3 * g1 + 1] - s[L.gxpos + 3 * g2 + 1],
                         s[L.gxpos + 3 * g1 + 2] - s[L.gxpos + 3 * g2 + 2]};
    const float rb = m.geom_rbound[g1] + m.geom_rbound[g2] + m.pair_margin[p];
    return dot3(dv, dv) <= rb * rb;
  };
  // one round: lane's pair p (-1: none) through the narrowphase when `cand`, then the group's contacts
  // appended in lane order (= pair order)
  auto pair_round = [&](int p, bool cand) {
    gCon* c = (gCon*)(scr + S.stage) + kMaxPairCon * lane;  // per-lane staging in global scratch
    int n = 0;
    unsigned long long t_np = SUB_T();
    if (p >= 0 && cand) {
      const int g1 = m.pair_g1[p], g2 = m.pair_g2[p];
      const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
      float p1[3], p2[3], m1[9], m2[9];
      for (int i = 0; i < 3; ++i) { p1[i] = s[L.gxpos + 3 * g1 + i]; p2[i] = s[L.gxpos + 3 * g2 + i]; }
      for (int i = 0; i < 9; ++i) { m1[i] = s[L.gxmat + 9 * g1 + i]; m2[i] = s[L.gxmat + 9 * g2 + i]; }
      float s1[3] = {m.geom_size[3 * g1], m.geom_size[3 * g1 + 1], m.geom_size[3 * g1 + 2]};
      float s2[3] = {m.geom_size[3 * g2], m.geom_size[3 * g2 + 1], m.geom_size[3 * g2 + 2]};
      n = narrowphase<G>(m, t1, t2, p1, m1, s1, p2, m2, s2, m.pair_margin[p], c, s + L.gxpos, s + L.gxmat, m.geom_size, g1, g2);
    }
    SUB_ADD(PH_COLL_NARROW, t_np);
    unsigned long long t_out = SUB_T();
    int total;
    static_assert(kMaxPairCon < 16, "contacts per pair must fit the 4-bit scan");
    int off = gscan_excl_small<G, 4>(n, total);  // (n <= kMaxPairCon = 8)
    if constexpr (G == 64) {
      // the next staged contact is loaded before this one's record is stored: a staging load issued
      // after a store would wait for it (vmcnt counts stores too), one store round trip per contact
      // of a box-box face polygon
      auto ld = [&](int k) {
        Con o;
        const gfloat* cf = (const gfloat*)(c + k);
        o.dist = cf[0];
        for (int i = 0; i < 3; ++i) { o.pos[i] = cf[1 + i]; o.nrm[i] = cf[4 + i]; }
        return o;
      };
      Con nx = ld(0);
      #pragma unroll 1
      for (int k = 0; k < n; ++k) {
        const Con cur = nx;
        nx = ld(k + 1 < kMaxPairCon ? k + 1 : k);
        const int slot = ncon + off + k;
        if (slot >= m.max_con) break;
        // (words 14, 15 are the rows phase's; written here only to make four 16-byte stores)
        __attribute__((address_space(1))) v4f* rec = (__attribute__((address_space(1))) v4f*)(scr + S.con + kConRec * slot);
        float fr[9] = {cur.nrm[0], cur.nrm[1], cur.nrm[2], 0, 0, 0, 0, 0, 0};
        make_frame(fr);
        rec[0] = (v4f){__int_as_float(p), cur.dist, cur.pos[0], cur.pos[1]};
        rec[1] = (v4f){cur.pos[2], fr[0], fr[1], fr[2]};
        rec[2] = (v4f){fr[3], fr[4], fr[5], fr[6]};
        rec[3] = (v4f){fr[7], fr[8], 0.0f, 0.0f};
      }
    } else {
      #pragma unroll 1
      for (int k = 0; k < n; ++k) {
        const int slot = ncon + off + k;
        if (slot >= m.max_con) break;
        gfloat* rec = scr + S.con + kConRec * slot;
        float fr[9] = {c[k].nrm[0], c[k].nrm[1], c[k].nrm[2], 0, 0, 0, 0, 0, 0};
        make_frame(fr);
        rec[0] = __int_as_float(p);
        rec[1] = c[k].dist;
        for (int i = 0; i < 3; ++i) rec[2 + i] = c[k].pos[i];
        for (int i = 0; i < 9; ++i) rec[5 + i] = fr[i];
      }
    }
    ncon += total;
    SUB_ADD(PH_COLL_OUT, t_out);
  };
  if (G == 64 && m.npair <= kCandPairs && !(m.diag_skip & 8)) {  // (MRS_DIAG_SKIP bit 3: pair-by-pair rounds, A/B)
    // candidates compacted first: the sphere tests of every pair as ballot bits (kCandPairs / 32
    // words per lane, the group's bits), then rounds of G candidates in pair order -- the
    // narrowphase's type branches run once per G candidates instead of once per G pairs, most of
    // which the sphere test rejects.  Measured (MRS_DIAG_SKIP=8 A/B, same box): C5 8.39 vs 8.48 ms
    // per launch; with lane groups C3 0.448 vs 0.446 ms (more scratch in its frame) and C4 equal,
    // so lane groups keep the pair-by-pair rounds
    constexpr int kW = kCandPairs / 32;
    unsigned cw[kW];
    unroll<kW>([&](auto wc) { cw[decltype(wc)::value] = 0u; });
    unroll<kCandPairs / G>([&](auto pc) {
      constexpr int q = decltype(pc)::value;
      if (q * G < m.npair) {
        const int p = q * G + lane;
        const bool cand = p < m.npair && sphere_cand(p);
        const unsigned long long bal = __ballot(cand);
        const unsigned bits = static_cast<unsigned>((bal >> (__lane_id() & ~(G - 1))) & ((G == 64) ? ~0ull : ((1ull << G) - 1)));
        if constexpr (G == 64) {
          cw[2 * q] = static_cast<unsigned>(bal);
          cw[2 * q + 1] = static_cast<unsigned>(bal >> 32);
        } else {
          cw[(q * G) / 32] |= bits << ((q * G) % 32);
        }
      }
    });
    int ncand = 0;
    unroll<kW>([&](auto wc) { ncand += __builtin_popcount(cw[decltype(wc)::value]); });
    const int rounds = uniform_int(wave_max((ncand + G - 1) / G));
    #pragma unroll 1
    for (int r = 0; r < rounds; ++r) {
      // this lane's candidate: the n-th set bit over the words (binary search by popcounts)
      int n = r * G + lane, p = -1;
      unroll<kW>([&](auto wc) {
        constexpr int w = decltype(wc)::value;
        const unsigned x0 = cw[w];
        const int pc = __builtin_popcount(x0);
        if (p < 0 && n >= 0 && n < pc) {
          unsigned x = x0;
          int pos = 0;
          int c = __builtin_popcount(x & 0xffffu); if (n >= c) { n -= c; x >>= 16; pos += 16; }
          c = __builtin_popcount(x & 0xffu); if (n >= c) { n -= c; x >>= 8; pos += 8; }
          c = __builtin_popcount(x & 0xfu); if (n >= c) { n -= c; x >>= 4; pos += 4; }
          c = __builtin_popcount(x & 0x3u); if (n >= c) { n -= c; x >>= 2; pos += 2; }
          c = static_cast<int>(x & 1u); if (n >= c) { pos += 1; }
          p = 32 * w + pos;
        }
        n -= pc;
      });
      pair_round(p, true);
    }
  } else {
    #pragma unroll 1
    for (int base = 0; base < m.npair; base += G) {
      const int p = base + lane;
      pair_round(p < m.npair ? p : -1, p < m.npair && sphere_cand(p));
    }
  }
  if (ncon > m.max_con) ncon = m.max_con;
  wsync();
  return ncon;
}

// acc + a * (v of lane K of the row): one v_fmac_f32 with the row broadcast as its DPP source
// operand (the compiler keeps a separate v_mov_dpp).  The s_nop covers the two wait states a DPP read
// of a VGPR needs after the VALU write that produced it (the hazard recognizer does not see inside
// inline asm).  The recognizer does not see the asm's own writes either, so a compiler-placed DPP
// read of the result within two instructions after it would miss its wait states: no such read occurs
// (tests/test_kernel_code.py checks the built kernels' disassembly; a trailing s_nop in the asm cost
// C5 2.8 % in the sweep).
template <int K>
__device__ __forceinline__ float fmac_rowb(float acc, float a, float v) {
  asm("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
               : "+v"(acc) : "v"(v), "v"(a), "n"(K));
  return acc;
}
// three held rows at once, the chain's own first: a += x * b, c += x * d, e += x * f with x lane K's
// v (every update a v_fmac_f32 with the broadcast as its DPP operand, one wait for all three)
template <int K>
__device__ __forceinline__ void fmac3_rowb(float& g0, float& g1, float& g2, float v, float a0, float a1, float a2) {
  asm("s_nop 1\n\t"
      "v_fmac_f32_dpp %0, %3, %4 row_newbcast:%7 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %1, %3, %5 row_newbcast:%7 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_fmac_f32_dpp %2, %3, %6 row_newbcast:%7 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "+v"(g0), "+v"(g1), "+v"(g2) : "v"(v), "v"(a0), "v"(a1), "v"(a2), "n"(K));
}
// v = own on lanes O, O + 16, O + 32, O + 48 (slot O of every 16-lane pipe), other elsewhere: one
// v_cndmask with a constant lane mask (no per-use compare)
template <int O>
__device__ __forceinline__ float sel_slot16(float own, float other) {
  constexpr unsigned long long mask = 0x0001000100010001ull << O;
  float r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(other), "v"(own), "s"(mask));
  return r;
}
// mj_makeConstraint + mj_makeImpedance + PGS (matrix-free rows) -> qacc, qfrc_constraint
// Small constraint systems on G = 16 groups (nv <= 16, nefc <= 16): lane j holds column j of J and
// of M^-1 J' for every row (registers, rows unrolled), row scalars are replicated in every lane of
// the group, row broadcasts are DPP row_newbcast and dot products DPP row reductions, so warm start
// and the PGS sweeps touch no memory.  Inputs: the dense rows J (global scratch, row-major) and,
// in lane r, row r's R, aref, b and friction-loss bound (0 for unilateral rows).  Returns qacc of
// lane j's dof and writes qfrc_constraint.  Rows past the group's nefc (up to the wave's maximum)
// are zero rows with R = 1, which never move.
// kUnit: every row's Jacobian is the unit vector of the dof held in lane r's `mydof` (dof friction
// loss rows), built in registers instead of read from the global rows J
// KV: the dof loops' unroll bound (>= nv; the call site picks 8 or 16), separate from the row count
template <bool kUnit = false, int KR = 16, int KV = 16, bool kRegAR = false>
__device__ __forceinline__ float pgs_small16(const DevModel& m, lfloat* s, const gfloat* J, gfloat* ff, int nefc, int rmax,
                                             float myR, float myaref, float myb, float myfl, float qacc_s,
                                             int lane, int mydof = -1) {
  const LdsLayout& L = m.L;
  const int nv = m.nv;
  // instantiated per row count KR (the wave's rmax rounded up to 4 at the call site): rows past the
  // wave's own are zero rows, so every row loop runs to the compile-time KR without bound tests
  rmax = KR;
  unsigned long long t_p = SUB_T();  // (timing builds: set-up / Delassus / warm start / sweeps)
  // J and M^-1 J' columns per row in registers; row scalars (R, aref, b, bound, diagonal of A, force)
  // stay in the row's own lane and reach the other lanes by DPP row broadcasts when used
  float Jt[KR], MJt[KR];
  if (lane >= nefc) { myR = 1; myaref = 0; myb = 0; myfl = 0; }
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (kUnit)
      Jt[r] = (r < nefc && lane == __float_as_int(rowb<r>(__int_as_float(mydof)))) ? 1.0f : 0.0f;
    else
      Jt[r] = (r < nefc && lane < nv) ? J[r * nv + lane] : 0.0f;
    MJt[r] = Jt[r];
  });
  // M^-1 J' for all rows at once: forward then backward substitution with L (Cholesky of M, LDS)
  unroll<KV>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if (i < nv) {
      const float inv = 1.0f / s[L.L + i * nv + i];
      const float lji = (lane > i && lane < nv) ? s[L.L + lane * nv + i] : 0.0f;
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if (r < rmax) {
          const float xi = rowb<i>(MJt[r]) * inv;
          MJt[r] = lane == i ? xi : MJt[r] - lji * xi;
        }
      });
    }
  });
  unroll<KV>([&](auto ic) {
    constexpr int i = KV - 1 - decltype(ic)::value;
    if (i < nv) {
      const float inv = 1.0f / s[L.L + i * nv + i];
      const float lij = lane < i ? s[L.L + i * nv + lane] : 0.0f;
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if (r < rmax) {
          const float zi = rowb<i>(MJt[r]) * inv;
          MJt[r] = lane == i ? zi : MJt[r] - lij * zi;
        }
      });
    }
  });
  SUB_ADD(PH_REC_SOLVE, t_p);
  t_p = SUB_T();
  // Delassus rows (mj_solPGS's efc_AR): lane r holds AR_rs = J_r M^-1 J_s' (+ R_r on the diagonal)
  // for every s; each (r, s <= r) product is one group sum, mirrored into lane s
  float AR[KR];
  float myA = 1, myf = 0;  // lane r: A_rr and the force of row r
  unroll<KR>([&](auto rc) { AR[decltype(rc)::value] = 0.0f; });
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    unroll<r + 1>([&](auto sc) {
      constexpr int c = decltype(sc)::value;
      if (r < rmax) {
        const float a = gsum<16>(Jt[r] * MJt[c]);
        // kRegAR: selects, not conditional stores -- the compiler merges the two conditional stores
        // into one store through a selected address, which keeps AR in a scratch array.  In registers
        // the out-of-line dense path clobbers more of its caller's registers, which the kernels where
        // it is cold (C2, C3) pay for in spills around their hot loop; where it is hot (the helper-wave
        // kernel, C4's contacts every step) the register form is the faster one
        if constexpr (kRegAR) {
          if constexpr (c == r) {
            AR[r] = lane == r ? a + myR : AR[r];
            myA = lane == r ? AR[r] : myA;
          } else {
            AR[c] = lane == r ? a : AR[c];
            AR[r] = lane == c ? a : AR[r];
          }
        } else {
          if constexpr (c == r) {
            if (lane == r) { AR[r] = a + myR; myA = AR[r]; }
          } else {
            if (lane == r) AR[c] = a;
            if (lane == c) AR[r] = a;
          }
        }
      }
    });
  });
  SUB_ADD(PH_CON_DEL, t_p);
  t_p = SUB_T();
  // warm start: forces of mj_constraintUpdate at qacc_warmstart, kept if the dual cost
  // f' (0.5 AR f + b) is negative.  Lane r owns row r: it alone computes the row's force, which every
  // lane then takes from it by broadcast
  if (!(m.disableflags & MRS_DSBL_WARMSTART)) {
    const float qw = lane < nv ? s[L.qacc_ws + lane] : 0.0f;
    float myjar = 0;
    unroll<KR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if (r < rmax) {
        const float jr = gsum<16>(Jt[r] * qw);
        if (lane == r) myjar = jr - myaref;
      }
    });
    {
      const float D = 1.0f / myR;
      myf = lane >= nefc ? 0.0f
                         : (myfl > 0 ? (myjar <= -myR * myfl ? myfl : (myjar >= myR * myfl ? -myfl : -D * myjar))
                                     : (myjar < 0 ? -D * myjar : 0.0f));
    }
    float arf = 0;
    unroll<KR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if (r < rmax) arf += AR[r] * rowb<r>(myf);
    });
    const float cost = gsum<16>(lane < rmax ? myf * (0.5f * arf + myb) : 0.0f);
    if (cost > 0) myf = 0;
  }
  // PGS sweeps on the dual (mj_solPGS): forces replicated in every lane; lane t keeps the residual
  // g_t = b_t + sum_s AR_ts f_s (computed once, then moved by AR_tr delta_r after row r's update), so
  // a row costs one broadcast of its residual and one FMA per lane instead of a group reduction of
  // J_r qacc.  Lane r also keeps row r's residual and step of the sweep; the sweep's cost improvement
  // sum_r -(delta_r res_r + 0.5 A_rr delta_r^2) (every term >= 0) is one group sum at its end.
  // The sweeps carry, in lane t, the normalised residual gn_t = -g_t / A_tt of its own row and the
  // normalised column ARn[r] = -AR_tr / A_tt (as the island-dual solver, constraints_sparse): row r's
  // step is the owner's med3 of its own gn (no broadcast on the chain), and every lane moves by
  // ARn[r] times that step with the DPP row broadcast folded into the FMA (fmac_rowb) -- a row is
  // med3 -> fmac_dpp on the chain instead of broadcast-multiply -> med3 -> FMA.  The owner's bounds
  // (lo - f, hi - f) move only at its own level, so they are updated after the sweep from the
  // residual it kept there (gb), with the sweep's improvement.
  float g;
  {
    float ga = lane < rmax ? myb : 0.0f, gb = 0, gc = 0, gd = 0;
    unroll<KR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if (r < rmax) {
        float& acc = (r & 3) == 0 ? ga : (r & 3) == 1 ? gb : (r & 3) == 2 ? gc : gd;
        acc += AR[r] * rowb<r>(myf);
      }
    });
    g = (ga + gb) + (gc + gd);
  }
  const float nia = -1.0f / myA;
  float gn = nia * g, ARn[KR];
  unroll<KR>([&](auto rc) { ARn[decltype(rc)::value] = nia * AR[decltype(rc)::value]; });
  float mylo = (myfl > 0 ? -myfl : 0.0f) - myf, myhi = (myfl > 0 ? myfl : __builtin_inff()) - myf;
  int nit = 0;  // sweeps done (mjData.solver_niter)
  SUB_ADD(PH_CON_WARM, t_p);
  t_p = SUB_T();
  // the sweep is unrolled to the wave's row count rounded up to 4 (rows past rmax are the zero rows,
  // which never move): no per-row bound tests inside the sweep
  auto sweeps = [&](auto nc) {
    constexpr int N = decltype(nc)::value;
    #pragma unroll 1
    for (int it = 0; it < m.iterations; ++it) {
      float gb = gn;
      unroll<N>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        const float cand = __builtin_amdgcn_fmed3f(gn, mylo, myhi);  // row r's clamped step, in lane r
        gb = sel_slot16<r>(gn, gb);
        gn = fmac_rowb<r>(gn, ARn[r], cand);
      });
      const float dm = __builtin_amdgcn_fmed3f(gb, mylo, myhi);
      mylo -= dm;
      myhi -= dm;
      const float improvement = gsum<16>(lane < rmax ? myA * dm * (gb - 0.5f * dm) : 0.0f);
      nit = it + 1;
      if (improvement * m.pgs_scale < m.tolerance) break;
    }
  };
  if (KR <= 4 || rmax <= 4) sweeps(std::integral_constant<int, (KR < 4 ? KR : 4)>{});
  else if (KR <= 8 || rmax <= 8) sweeps(std::integral_constant<int, (KR < 8 ? KR : 8)>{});
  else if (KR <= 12 || rmax <= 12) sweeps(std::integral_constant<int, (KR < 12 ? KR : 12)>{});
  else sweeps(std::integral_constant<int, KR>{});
  SUB_ADD(PH_REC_ROWS, t_p);
  myf = (myfl > 0 ? -myfl : 0.0f) - mylo;
  float f[KR];
  unroll<KR>([&](auto rc) { f[decltype(rc)::value] = rowb<decltype(rc)::value>(myf); });
  float qa = lane < nv ? qacc_s : 0.0f;  // qacc = qacc_smooth + M^-1 J' f
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if (r < rmax) qa += MJt[r] * f[r];
  });
  if (lane == 0) s[L.niter] = __int_as_float(nit);
  float qc = 0;
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if (r < rmax) qc += Jt[r] * f[r];
  });
  if (lane < nv) s[L.qfrc_con + lane] = qc;
  // row forces (mj_rnePostConstraint's contact forces, mrs_batch_get_efc)
  // (the friction-loss fast path stores them only when force/torque sensors read them)
  if (ff && (!kUnit || (m.acc_sens & 2)) && lane < nefc) ff[lane] = myf;
  return qa;
}

// The same PGS in qacc form (each row's residual is a group sum of J_r qacc): used for the
// friction-loss unit rows, whose systems converge in a few sweeps, where the dual form's O(rows^2)
// Delassus set-up costs more than its shorter sweep chain saves (C3: 179 vs 171 M env-steps/s)
template <bool kUnit = false, int KR = 16>
__device__ __forceinline__ float pgs_small16_qacc(const DevModel& m, lfloat* s, const gfloat* J, gfloat* ff, int nefc, int rmax,
                                             float myR, float myaref, float myb, float myfl, float qacc_s,
                                             int lane, int mydof = -1, unsigned fmask = 0) {
  const LdsLayout& L = m.L;
  const int nv = m.nv;
  // kUnit (dof friction-loss rows): row r is the unit vector of dof r, held in lane r (rows indexed by
  // dof, the bit of fmask says whether dof r has a row; mydof is then the lane's row index in the
  // efc order, for the row forces).  J_r x is then lane r's x -- a DPP broadcast or nothing, not a
  // group reduction -- and the rows keep mj_makeConstraint's order (dof order).
  const bool myrow = kUnit ? ((fmask >> lane) & 1u) != 0 : lane < nefc;
  // J and M^-1 J' columns per row in registers; row scalars (R, aref, b, bound, diagonal of A, force)
  // stay in the row's own lane and reach the other lanes by DPP row broadcasts when used
  float Jt[KR], MJt[KR];
  if (!myrow) { myR = 1; myaref = 0; myb = 0; myfl = 0; }
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (kUnit)
      Jt[r] = (lane == r && ((fmask >> r) & 1u)) ? 1.0f : 0.0f;
    else
      Jt[r] = (r < nefc && lane < nv) ? J[r * nv + lane] : 0.0f;
    MJt[r] = Jt[r];
  });
  // M^-1 J' for all rows at once: forward then backward substitution with L (Cholesky of M, LDS)
  unroll<KR>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    if (i < nv) {
      const float inv = 1.0f / s[L.L + i * nv + i];
      const float lji = (lane > i && lane < nv) ? s[L.L + lane * nv + i] : 0.0f;
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if (r < rmax) {
          const float xi = rowb<i>(MJt[r]) * inv;
          MJt[r] = lane == i ? xi : MJt[r] - lji * xi;
        }
      });
    }
  });
  unroll<KR>([&](auto ic) {
    constexpr int i = KR - 1 - decltype(ic)::value;
    if (i < nv) {
      const float inv = 1.0f / s[L.L + i * nv + i];
      const float lij = lane < i ? s[L.L + i * nv + lane] : 0.0f;
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if (r < rmax) {
          const float zi = rowb<i>(MJt[r]) * inv;
          MJt[r] = lane == i ? zi : MJt[r] - lij * zi;
        }
      });
    }
  });
  float myA = 1, myf = 0;  // lane r: A_rr = J_r M^-1 J_r' + R_r and the force of row r
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (kUnit) {
      if (lane == r) myA = MJt[r] + myR;  // (M^-1)_rr + R_r, in lane r itself
    } else if (r < rmax) {
      const float a = gsum<16>(Jt[r] * MJt[r]) + rowb<r>(myR);
      if (lane == r) myA = a;
    }
  });
  float qa = lane < nv ? qacc_s : 0.0f;
  // warm start: forces of mj_constraintUpdate at qacc_warmstart, kept if the dual cost is negative.
  // Lane r owns row r: it alone computes the row's force, which every lane then takes from it by
  // broadcast, so M^-1 J' f and the sweeps' forces are built from one value per row
  if (!(m.disableflags & MRS_DSBL_WARMSTART)) {
    const float qw = lane < nv ? s[L.qacc_ws + lane] : 0.0f;
    float myjar = 0;
    if constexpr (kUnit) {
      myjar = qw - myaref;
    } else {
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if (r < rmax) {
          const float jr = gsum<16>(Jt[r] * qw);
          if (lane == r) myjar = jr - myaref;
        }
      });
    }
    {
      const float D = 1.0f / myR;
      myf = !myrow ? 0.0f
                         : (myfl > 0 ? (myjar <= -myR * myfl ? myfl : (myjar >= myR * myfl ? -myfl : -D * myjar))
                                     : (myjar < 0 ? -D * myjar : 0.0f));
    }
    float v = 0;
    unroll<KR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if (r < rmax) v += MJt[r] * rowb<r>(myf);
    });
    float cost = 0;
    if constexpr (kUnit) {
      cost = gsum<16>(myrow ? myf * (0.5f * (v + myR * myf) + myb) : 0.0f);
    } else {
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        if (r < rmax) {
          const float f = rowb<r>(myf);
          cost += f * (0.5f * (gsum<16>(Jt[r] * v) + rowb<r>(myR) * f) + rowb<r>(myb));
        }
      });
    }
    if (cost > 0) {
      myf = 0;
    } else {
      qa += v;
    }
  }
  // PGS sweeps: row scalars broadcast into every lane once, forces replicated across the sweeps
  float f[KR], bR[KR], bA[KR], iA[KR], bref[KR], bfl[KR];
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    f[r] = rowb<r>(myf); bR[r] = rowb<r>(myR); bA[r] = rowb<r>(myA); bref[r] = rowb<r>(myaref);
    bfl[r] = rowb<r>(myfl); iA[r] = 1.0f / bA[r];
  });
  int nit = 0;  // sweeps done (mjData.solver_niter)
  #pragma unroll 1
  for (int it = 0; it < m.iterations; ++it) {
    float improvement = 0;
    unroll<KR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if (kUnit ? ((fmask >> r) & 1u) != 0 : r < rmax) {
        const float res = (kUnit ? rowb<r>(qa) : gsum<16>(Jt[r] * qa)) - bref[r] + bR[r] * f[r];
        float nf = f[r] - res * iA[r];
        nf = bfl[r] > 0 ? clampf(nf, -bfl[r], bfl[r]) : (nf < 0 ? 0.0f : nf);
        const float delta = nf - f[r];
        qa += MJt[r] * delta;
        f[r] = nf;
        improvement -= delta * res + 0.5f * delta * delta * bA[r];
      }
    });
    nit = it + 1;
    if (improvement * m.pgs_scale < m.tolerance) break;
  }
  if (lane == 0) s[L.niter] = __int_as_float(nit);
  float qc = 0;
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (kUnit) {
      if (lane == r) qc = Jt[r] * f[r];
    } else if (r < rmax) {
      qc += Jt[r] * f[r];
    }
    if (lane == r) myf = f[r];
  });
  if (lane < nv) s[L.qfrc_con + lane] = qc;
  // row forces (mj_rnePostConstraint's contact forces, mrs_batch_get_efc; kUnit: at the row's efc
  // index, only when force/torque sensors read them)
  if (ff && (!kUnit || (m.acc_sens & 2)) && myrow) ff[kUnit ? mydof : lane] = myf;
  return qa;
}

// ---------------------------------------------------------------- blocked mode: sparse rows
// One env per wave (G = 64).  M is block diagonal over kinematic trees and a constraint row touches
// at most two trees, so each row is stored over the dof slots of its trees only: P = pipe_w slots,
// 64 / P rows in flight per wave ("pipes").  Rows are grouped into islands (trees connected through
// contacts, as mj_island); rows of different islands share no dof, so the Gauss-Seidel sweeps of
// different islands commute and each pipe sweeps its own islands in row order -- the same PGS
// iterates as the row-serial solver (mj_solPGS), 64 / P rows per step instead of one.  Islands go to
// pipes by longest-processing-time.  Records (J, M^-1 J' and dof per slot, row scalars) sit in the
// env's scratch in solver order, pipe p's rows at [start_p, start_p + n_p); each level k of a sweep
// is one row per pipe, its record prefetched a level ahead; qacc and the row forces stay in LDS.
constexpr int kHdr = 24;     // item header floats (blocked mode; batch.hip sizes efc_hdr to match)
constexpr int kRecScal = 12;  // aref, R, ARii, bound (frictionloss, -1 otherwise), b, then the coupling
                              // J_r M^-1 J_s' of row r to the earlier rows s < r of its item (3 floats),
                              // J qacc_warmstart - aref, 3 pad
#ifndef MRS_REG_QUADS
#define MRS_REG_QUADS 12
#endif
constexpr int kRegQuads = MRS_REG_QUADS;  // items per pipe of the item-blocked register solve
#ifndef MRS_REG_LEVELS
#define MRS_REG_LEVELS 48
#endif
constexpr int kRegLevels = MRS_REG_LEVELS;  // rows per pipe of the register-resident solve
#ifndef MRS_DUAL_LEVELS
#define MRS_DUAL_LEVELS 48
#endif
constexpr int kDualLevels = MRS_DUAL_LEVELS;  // rows per pipe of the island-dual register solve (x16)

__device__ __forceinline__ int slot_dof(const DevModel& m, int t1, int t2, int slot) {
  if (t1 < 0) return -1;
  const int n1 = m.tree_dofnum[t1];
  if (slot < n1) return m.tree_dofadr[t1] + slot;
  if (t2 < 0) return -1;
  const int l2 = slot - n1;
  return l2 < m.tree_dofnum[t2] ? m.tree_dofadr[t2] + l2 : -1;
}
// a tree's (dofadr, dofnum, M block offset) from the env's LDS copy of the tree table
struct TreeInfo { int adr, num, off; };
__device__ __forceinline__ TreeInfo tree_lds(const lfloat* s, const LdsLayout& L, int t) {
  const v4f v = *(const __attribute__((address_space(3))) v4f*)(s + L.trees + 4 * (t < 0 ? 0 : t));
  return TreeInfo{__float_as_int(v.x), t < 0 ? 0 : __float_as_int(v.y), __float_as_int(v.z)};
}
// slot -> (dof, tree segment) of a row over trees t1, t2 (LDS tree table)
struct SlotMap { int d, li, n, off, sb; };
__device__ __forceinline__ SlotMap slot_map(const lfloat* s, const LdsLayout& L, int t1, int t2, int slot) {
  const TreeInfo a = tree_lds(s, L, t1), b = tree_lds(s, L, t2);
  SlotMap r{-1, 0, 0, 0, 0};
  if (t1 >= 0 && slot < a.num) { r.d = a.adr + slot; r.li = slot; r.n = a.num; r.off = a.off; }
  else if (t1 >= 0 && t2 >= 0 && slot - a.num < b.num) { r.d = b.adr + slot - a.num; r.li = slot - a.num; r.n = b.num; r.off = b.off; r.sb = a.num; }
  return r;
}
// slot -> (dof, tree segment) in an island's frame: its trees (packed t + 1 per byte, tree order) laid
// out one after the other
__device__ __forceinline__ SlotMap island_slot_map(const lfloat* s, const LdsLayout& L, unsigned pack, int slot) {
  SlotMap r{-1, 0, 0, 0, 0};
  int base = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int t = static_cast<int>((pack >> (8 * q)) & 0xffu) - 1;
    if (t >= 0) {
      const TreeInfo ti = tree_lds(s, L, t);
      if (r.d < 0 && slot >= base && slot < base + ti.num) { r.d = ti.adr + slot - base; r.li = slot - base; r.n = ti.num; r.off = ti.off; r.sb = base; }
      base += ti.num;
    }
  }
  return r;
}
// trees of a row from its descriptor: t1 >= 0 unless the row touches no dof; t2 = -1 for one tree
__device__ __forceinline__ void row_trees(const DevModel& m, const gfloat* scr, int code, int& t1, int& t2) {
  const int t = code >> 16, id = code & 0xffff;
  t2 = -1;
  if (t == EFC_FRICTION) {
    t1 = m.dof_tree[id];
  } else if (t == EFC_LIMIT) {
    t1 = m.dof_tree[m.jnt_dofadr[id]];
  } else {
    const int p = __float_as_int(scr[m.S.con + kConRec * id]);
    int a = m.body_tree[m.geom_bodyid[m.pair_g1[p]]], b = m.body_tree[m.geom_bodyid[m.pair_g2[p]]];
    if (a < 0) { a = b; b = -1; }
    if (b == a) b = -1;
    t1 = a;
    t2 = b;
  }
}
// x = M^-1 v restricted to the row's trees; the P slot lanes of one pipe hold v.  Block-wise forward
// and back substitution; the pivot of step k of a tree segment is the segment's lane k.
__device__ __forceinline__ float pipe_msolve(const DevModel& m, const lfloat* Lf, int t1, int t2, int slot, int pbase,
                                             float v) {
  int tr = -1, li = 0, sb = 0;
  const int n1 = t1 >= 0 ? m.tree_dofnum[t1] : 0;
  if (t1 >= 0 && slot < n1) { tr = t1; li = slot; }
  else if (t2 >= 0 && slot - n1 < m.tree_dofnum[t2]) { tr = t2; li = slot - n1; sb = n1; }
  const int n = tr >= 0 ? m.tree_dofnum[tr] : 0;
  const lfloat* Lb = Lf + (tr >= 0 ? m.tree_Moff[tr] : 0);
  float x = tr >= 0 ? v : 0.0f;
  const int src = pbase + sb;
  #pragma unroll 1
  for (int k = 0; k < m.tree_nmax; ++k) {
    const float xs = __shfl(x, src + k);
    if (k < n) {
      const float xk = xs / Lb[k * n + k];
      if (li == k) x = xk;
      else if (li > k) x -= Lb[li * n + k] * xk;
    }
  }
  #pragma unroll 1
  for (int k = m.tree_nmax - 1; k >= 0; --k) {
    const float xs = __shfl(x, src + k);
    if (k < n) {
      const float xk = xs / Lb[k * n + k];
      if (li == k) x = xk;
      else if (li < k) x -= Lb[k * n + li] * xk;
    }
  }
  return x;
}
// three right-hand sides at once (a contact's normal and tangent Jacobian rows): the substitution
// chains interleave and share the pivot reciprocal
__device__ __forceinline__ void pipe_msolve3(const DevModel& m, const lfloat* Lf, const SlotMap& sm, int pbase,
                                             const float v[3], float x[3]) {
  const int li = sm.li, n = sm.n;
  const lfloat* Lb = Lf + sm.off;
  for (int i = 0; i < 3; ++i) x[i] = sm.d >= 0 ? v[i] : 0.0f;
  const int src = pbase + sm.sb;
  #pragma unroll 1
  for (int k = 0; k < m.tree_nmax; ++k) {
    float xs[3];
    for (int i = 0; i < 3; ++i) xs[i] = __shfl(x[i], src + k);
    if (k < n) {
      const float inv = 1.0f / Lb[k * n + k];
      const float lik = li > k ? Lb[li * n + k] : 0.0f;
      for (int i = 0; i < 3; ++i) {
        const float xk = xs[i] * inv;
        x[i] = li == k ? xk : (li > k ? x[i] - lik * xk : x[i]);
      }
    }
  }
  #pragma unroll 1
  for (int k = m.tree_nmax - 1; k >= 0; --k) {
    float xs[3];
    for (int i = 0; i < 3; ++i) xs[i] = __shfl(x[i], src + k);
    if (k < n) {
      const float inv = 1.0f / Lb[k * n + k];
      const float lki = li < k ? Lb[k * n + li] : 0.0f;
      for (int i = 0; i < 3; ++i) {
        const float xk = xs[i] * inv;
        x[i] = li == k ? xk : (li < k ? x[i] - lki * xk : x[i]);
      }
    }
  }
}
// y = L^-1 v, the forward half of pipe_msolve3.  With M = L L' per tree, a row's record holds
// Y = L^-1 J' over its slots only: J_r M^-1 J_s' = Y_r . Y_s, and the solvers that track qacc work on
// w = L' qacc instead (J qacc = Y . w, and a force step df moves w by Y df); tree_epilogue maps back.
__device__ __forceinline__ void pipe_lsolve3(const DevModel& m, const lfloat* Lf, const SlotMap& sm, int pbase,
                                             const float v[3], float x[3]) {
  const int li = sm.li, n = sm.n;
  const lfloat* Lb = Lf + sm.off;
  for (int i = 0; i < 3; ++i) x[i] = sm.d >= 0 ? v[i] : 0.0f;
  const int src = pbase + sm.sb;
  #pragma unroll 1
  for (int k = 0; k < m.tree_nmax; ++k) {
    float xs[3];
    for (int i = 0; i < 3; ++i) xs[i] = __shfl(x[i], src + k);
    if (k < n) {
      const float inv = 1.0f / Lb[k * n + k];
      const float lik = li > k ? Lb[li * n + k] : 0.0f;
      for (int i = 0; i < 3; ++i) {
        const float xk = xs[i] * inv;
        x[i] = li == k ? xk : (li > k ? x[i] - lik * xk : x[i]);
      }
    }
  }
}
// Li = L^-1 per tree block (lane per dof d: column li(d) of its tree's inverse factor, forward
// substitution down the column; each lane reads only L and writes only its own column)
__device__ __forceinline__ void tree_linv(const DevModel& m, lfloat* s, const LdsLayout& L, int lane) {
  if (lane < m.nv) {
    const TreeInfo ti = tree_lds(s, L, m.dof_tree[lane]);
    const int n = ti.num, c = lane - ti.adr;
    const lfloat* Lb = s + L.L + ti.off;
    lfloat* Ib = s + L.Li + ti.off;
    Ib[c * n + c] = 1.0f / Lb[c * n + c];
    #pragma unroll 1
    for (int i = c + 1; i < n; ++i) {
      float acc = 0;
      #pragma unroll 1
      for (int k = c; k < i; ++k) acc += Lb[i * n + k] * Ib[k * n + c];
      Ib[i * n + c] = -acc / Lb[i * n + i];
    }
  }
  wsync();
}
// y = L^-1 v by the inverse factor (tree_linv): y_li = sum_k Li[li][k] v_k over the slot's tree
// segment, the v_k fetched from the segment's lanes by independent permutes (pipe_lsolve3's
// substitution is a dependent chain of one permute round trip per dof).  Segments of at most 8 dofs.
__device__ __forceinline__ void pipe_linv3(const lfloat* Li, const SlotMap& sm, int pbase, const float v[3], float x[3]) {
  const int li = sm.li, n = sm.n;
  const lfloat* Ib = Li + sm.off + li * n;
  const int src = pbase + sm.sb;
  float vv[3];
  for (int i = 0; i < 3; ++i) { vv[i] = sm.d >= 0 ? v[i] : 0.0f; x[i] = 0.0f; }
  unroll<8>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int sl = min(src + k, 63);
    float xs[3];
    for (int i = 0; i < 3; ++i) xs[i] = __shfl(vv[i], sl);
    const float lik = (sm.d >= 0 && k <= li) ? Ib[k] : 0.0f;
    for (int i = 0; i < 3; ++i) x[i] += lik * xs[i];
  });
}
// lane per dof (blocked mode, nv <= 64): the dof's tree segment in the LDS factor
struct DofTree { int adr, li, n; const lfloat* Lb; };
__device__ __forceinline__ DofTree dof_tree_lds(const DevModel& m, const lfloat* s, const LdsLayout& L, int lane) {
  DofTree r{0, 0, 0, s + L.L};
  if (lane < m.nv) {
    const TreeInfo ti = tree_lds(s, L, m.dof_tree[lane]);
    r.adr = ti.adr; r.li = lane - ti.adr; r.n = ti.num; r.Lb += ti.off;
  }
  return r;
}
// w = L' q per tree (lane per dof)
__device__ __forceinline__ float tree_lt_mul(const DevModel& m, const DofTree& t, float q) {
  float w = 0;
  #pragma unroll 1
  for (int k = 0; k < m.tree_nmax; ++k) {
    const float qk = __shfl(q, min(t.adr + k, 63));
    if (k >= t.li && k < t.n) w += t.Lb[k * t.n + t.li] * qk;
  }
  return w;
}
// sparse solver epilogue: z = sum_r Y_r f_r per dof in tmp -> qfrc_constraint = J' f = L z (written
// to tmp) and qacc = qacc_smooth + M^-1 J' f = qacc_smooth + L'^-1 z (written to qa and returned)
__device__ __forceinline__ float tree_epilogue(const DevModel& m, const lfloat* s, const LdsLayout& L, lfloat* tmp,
                                               lfloat* qa, float qacc_s, int lane) {
  const DofTree t = dof_tree_lds(m, s, L, lane);
  const float z = lane < m.nv ? tmp[lane] : 0.0f;
  float y = 0, acc = z, x = 0;
  #pragma unroll 1
  for (int k = 0; k < m.tree_nmax; ++k) {
    const float zk = __shfl(z, min(t.adr + k, 63));
    if (k <= t.li && k < t.n) y += t.Lb[t.li * t.n + k] * zk;
  }
  #pragma unroll 1
  for (int k = m.tree_nmax - 1; k >= 0; --k) {
    if (t.li == k && k < t.n) x = acc / t.Lb[k * t.n + k];
    const float xs = __shfl(x, min(t.adr + k, 63));
    if (k < t.n && t.li < k) acc -= t.Lb[k * t.n + t.li] * xs;
  }
  const float qacc = qacc_s + x;
  wsync();
  if (lane < m.nv) { tmp[lane] = y; qa[lane] = qacc; }
  wsync();
  return lane < m.nv ? qacc : 0.0f;
}
__device__ __forceinline__ int lanes_below(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(mask), 0));
}
// one record as the sweeps read it
template <int P>
struct RowRec {
  float Y, aref, R, a, bound;
  int d;
};
template <int P>
__device__ __forceinline__ RowRec<P> load_rec(const gfloat* rec, int q, int slot) {
  constexpr int RF = 2 * P + kRecScal;
  const gfloat* r = rec + q * RF;
  RowRec<P> o;
  o.Y = r[slot];
  o.d = __float_as_int(r[P + slot]);
  const v4f sc = *(const __attribute__((address_space(1))) v4f*)(r + 2 * P);
  o.aref = sc.x; o.R = sc.y; o.a = sc.z; o.bound = sc.w;
  return o;
}

template <int P>
__device__ float constraints_sparse(ENV_PARAMS, int ncon, float qacc_s) {
  constexpr int G = 64;
  ENV_UNPACK;
  ncon = uniform_int(ncon);
  constexpr int NP = 64 / P;
  constexpr int RF = 2 * P + kRecScal;
  const int pipe = lane / P, slot = lane % P, pbase = pipe * P;
  const int nv = m.nv, ME = m.max_efc;
  gfloat* type = scr + S.efc_type;
  gfloat* pos = scr + S.efc_pos;
  gfloat* marg = scr + S.efc_margin;
  gfloat* floss = scr + S.efc_floss;
  gfloat* rec = scr + S.efc_rec;
  gfloat* rowof = scr + S.efc_rowof;
  gfloat* ffg = scr + S.efc_f;
  gfloat* fl = scr + S.efc_fq;  // row forces by record position (global-record fallback path)
  lfloat* qa = s + L.qacc;      // qacc during the solve (lane per dof)
  lfloat* tmp = s + L.qfrc_con; // warm-start M^-1 J' f, then qfrc_constraint
  if (m.disableflags & MRS_DSBL_CONSTRAINT) { if (lane < nv) tmp[lane] = 0; wsync(); return qacc_s; }
  unsigned long long t_sub = SUB_T();

  // --- 1. row descriptors in the row-serial solver's order: friction loss, limits, contacts
  int nefc = 0;
  if (!(m.disableflags & MRS_DSBL_FRICTIONLOSS)) {
    #pragma unroll 1
    for (int r = lane; r < m.nfric; r += 64) {
      const int j = m.fric_dof[r];
      type[r] = __int_as_float(EFC_FRICTION * 65536 + j);
      pos[r] = 0; marg[r] = 0; floss[r] = m.dof_frictionloss[j];
    }
    nefc = m.nfric;
  }
  if (!(m.disableflags & MRS_DSBL_LIMIT)) {
    #pragma unroll 1
    for (int base = 0; base < m.nlim; base += 64) {
      const int k = base + lane;
      float dist[2] = {0, 0};
      int jid = -1;
      bool act[2] = {false, false};
      if (k < m.nlim) {
        jid = m.lim_jnt[k];
        const float q = s[L.qpos + m.jnt_qposadr[jid]], mg = m.jnt_margin[jid];
        dist[0] = q - m.jnt_range[2 * jid];
        dist[1] = m.jnt_range[2 * jid + 1] - q;
        act[0] = dist[0] < mg;
        act[1] = dist[1] < mg;
      }
      int total;
      int r = nefc + gscan_excl<64>((int)act[0] + (int)act[1], lane, total);
      for (int sd = 0; sd < 2; ++sd) {
        if (!act[sd]) continue;
        type[r] = __int_as_float(EFC_LIMIT * 65536 + jid);
        pos[r] = dist[sd];
        marg[r] = m.jnt_margin[jid];
        floss[r] = sd == 0 ? 1.0f : -1.0f;  // J sign
        ++r;
      }
      nefc += total;
    }
  }
  const int nsingle = nefc;  // friction-loss and limit rows: one item each
  #pragma unroll 1
  for (int base = 0; base < ncon; base += 64) {
    const int c = base + lane;
    gfloat* crec = scr + S.con + kConRec * (c < ncon ? c : 0);
    int nr = 0, p = 0;
    if (c < ncon) { p = __float_as_int(crec[0]); nr = m.pair_dim[p] == 1 ? 1 : 4; }
    int total;
    const int r0 = nefc + gscan_excl<64>(nr, lane, total);
    if (c < ncon) {
      crec[14] = __int_as_float(r0 + nr <= ME ? r0 : -1);
      crec[15] = __int_as_float(r0);
      for (int j = 0; j < nr; ++j) {
        const int r = r0 + j;
        if (r >= ME) break;
        type[r] = __int_as_float(EFC_CONTACT * 65536 + c);
        pos[r] = crec[1]; marg[r] = m.pair_margin[p] - m.pair_gap[p]; floss[r] = (float)j;
      }
    }
    nefc += total;
  }
  nefc = min(nefc, ME);
  wsync();
  if (nefc == 0) {
    if (lane < nv) tmp[lane] = 0;
    wsync();
    return qacc_s;
  }

  // --- 2. islands: lane t holds the smallest tree id of its component (contacts merge components)
  int lbl = lane;
  #pragma unroll 1
  for (int base = 0; base < ncon; base += 64) {
    const int c = base + lane;
    int a = -1, b = -1;
    if (c < ncon) {
      const int p = __float_as_int(scr[S.con + kConRec * c]);
      a = m.body_tree[m.geom_bodyid[m.pair_g1[p]]];
      b = m.body_tree[m.geom_bodyid[m.pair_g2[p]]];
    }
    const int nc = min(64, ncon - base);
    #pragma unroll 1
    for (int k = 0; k < nc; ++k) {
      const int ak = __builtin_amdgcn_readlane(a, k), bk = __builtin_amdgcn_readlane(b, k);
      if (ak < 0 || bk < 0 || ak == bk) continue;
      const int la = __builtin_amdgcn_readlane(lbl, ak), lb = __builtin_amdgcn_readlane(lbl, bk);
      const int lo = min(la, lb), hi = max(la, lb);
      if (lbl == hi) lbl = lo;
    }
  }
  // items: a friction-loss or limit row, or the consecutive 1 or 4 rows of one contact (rows past
  // max_efc are cut).  Rows per island (lane i: the island whose smallest tree is i); rows without
  // dofs go to pipe 0.
  const int nitem = nsingle + ncon;
  auto item_info = [&](int i, int& r0, int& nr) {
    if (i < nsingle) {
      r0 = i;
      nr = 1;
    } else {
      const gfloat* crec = scr + S.con + kConRec * (i - nsingle);
      r0 = __float_as_int(crec[15]);
      nr = max(0, min(m.pair_dim[__float_as_int(crec[0])] == 1 ? 1 : 4, ME - r0));
    }
  };
  auto wave_sum_int = [](int v) {
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
  };
  int cnt = 0, nodof = 0;
  #pragma unroll 1
  for (int base = 0; base < nitem; base += 64) {
    const int i = base + lane;
    int r0 = 0, nr = 0, t1 = -1, t2;
    if (i < nitem) item_info(i, r0, nr);
    if (nr > 0) row_trees(m, scr, __float_as_int(type[r0]), t1, t2);
    const int il = __shfl(lbl, t1 < 0 ? 0 : t1);
    nodof += wave_sum_int(t1 < 0 ? nr : 0);
    #pragma unroll 1
    for (int k = 0; k < m.ntree; ++k) {
      const int ck = wave_sum_int(t1 >= 0 && il == k ? nr : 0);
      if (lane == k) cnt += ck;
    }
  }
  // island slot frames: an island's trees in tree order, each tree's dofs consecutive (lane t: its
  // tree's slot offset `ioff` in its island; lane i: island i's dof count and up to 4 trees packed
  // (t + 1) per byte).  When every island with rows fits the pipe (<= P dofs, <= 4 trees), every row
  // of an island holds J and M^-1 J' over the same slots, so J_r M^-1 J_s' of any two rows of an
  // island is a plain slot-wise dot product (the dual solver's Delassus rows).
  int idof = 0, itr = 0;
  unsigned ipack = 0;
  #pragma unroll 1
  for (int k = 0; k < m.ntree; ++k) {
    const int lk = __builtin_amdgcn_readlane(lbl, k);
    if (lk == lane) {
      if (itr < 4) ipack |= static_cast<unsigned>(k + 1) << (8 * itr);
      ++itr;
      idof += m.tree_dofnum[k];
    }
  }
  const bool isl_ok = !__any(cnt > 0 && (idof > P || itr > 4));
  // longest-processing-time: largest island first onto the least loaded pipe
  int load[NP];
  unroll<NP>([&](auto pc) { load[decltype(pc)::value] = 0; });
  load[0] = nodof;
  int mypipe = 0;  // lane i: pipe of island i
  #pragma unroll 1
  for (;;) {
    const int key = wave_max(cnt > 0 ? (cnt << 8) | (255 - lane) : -1);
    if (key < 0) break;
    const int win = 255 - (key & 255), c = key >> 8;
    int best = 0, bl = load[0];
    unroll<NP>([&](auto pc) {
      constexpr int q = decltype(pc)::value;
      if (load[q] < bl) { bl = load[q]; best = q; }
    });
    if (lane == win) { mypipe = best; cnt = 0; }
    unroll<NP>([&](auto pc) {
      constexpr int q = decltype(pc)::value;
      if (q == best) load[q] += c;
    });
  }
  // solver order: pipe p's rows in row order at records [start_p, start_p + n_p)
  int start[NP], fill[NP], nlev = 0, my_n = 0, my_start = 0;
  {
    int acc = 0;
    unroll<NP>([&](auto pc) {
      constexpr int q = decltype(pc)::value;
      start[q] = acc; fill[q] = acc; acc += load[q];
      nlev = max(nlev, load[q]);
      if (pipe == q) { my_n = load[q]; my_start = start[q]; }
    });
    nlev = uniform_int(nlev);
  }
  gfloat* hdr = scr + S.efc_hdr;
  // item headers: everything the records phase needs that does not depend on the dof slot, computed
  // lane-per-item (64 items at once, no dependent chain per item there).  With at most 64 items
  // (C5: ~47) they stay in the item lane's registers and the records loop fetches its pipe's
  // current item by lane permute: no header round trip through the env's global scratch, whose
  // loads would wait (vmcnt counts stores too) for every record store issued before them.
  // Otherwise they go to the scratch (efc_hdr, kHdr floats at the item's first record).
  struct Hdr { v4f a, b, c, d, e, f; };
  const bool hreg = nitem <= 64;
  Hdr hv{};                       // hreg: this lane's item header (f.z: its first record)
  unsigned long long pend[NP];    // hreg: per pipe, the lanes of its items not yet built (item order)
  unroll<NP>([&](auto pc) { pend[decltype(pc)::value] = 0; });
  #pragma unroll 1
  for (int base = 0; base < nitem; base += 64) {
    const int i = base + lane;
    int r0 = 0, nr = 0, t1 = -1, t2;
    if (i < nitem) item_info(i, r0, nr);
    if (nr > 0) row_trees(m, scr, __float_as_int(type[r0]), t1, t2);
    const int il = __shfl(lbl, t1 < 0 ? 0 : t1);
    const int pr = t1 < 0 ? 0 : __shfl(mypipe, il);
    int q0 = 0;
    unroll<NP>([&](auto pc) {
      constexpr int q = decltype(pc)::value;
      int tot;
      const int ex = gscan_excl<64>(pr == q ? nr : 0, lane, tot);
      if (pr == q) q0 = fill[q] + ex;
      fill[q] += tot;
      if (hreg) pend[q] = __ballot(pr == q && nr > 0);
    });
    if (nr > 0) {
      const int code = __float_as_int(type[r0]);
      const int t = code >> 16, id = code & 0xffff;
      CPtr<float> sr, si;
      float diag, mu = 0, bound = -1;
      int dim = 1;
      if (t == EFC_FRICTION) {
        sr = m.dof_solref + 2 * id; si = m.dof_solimp + 5 * id; diag = m.dof_invweight0[id];
        bound = floss[r0];
      } else if (t == EFC_LIMIT) {
        sr = m.jnt_solref + 2 * id; si = m.jnt_solimp + 5 * id; diag = m.dof_invweight0[m.jnt_dofadr[id]];
      } else {
        const int p = __float_as_int(scr[S.con + kConRec * id]);
        dim = m.pair_dim[p];
        mu = m.pair_friction[3 * p];  // sliding, for both tangent directions
        sr = m.pair_solref + 2 * p; si = m.pair_solimp + 5 * p;
        const float tran = m.body_invweight0[2 * m.geom_bodyid[m.pair_g1[p]]] + m.body_invweight0[2 * m.geom_bodyid[m.pair_g2[p]]];
        // pyramid edges: diagApprox tran (1 + mu^2), regulariser scaled by 2 mu^2 / impratio
        // (mj_makeImpedance; oracle/oracle.c make_constraint)
        diag = dim == 3 ? tran * (1 + mu * mu) * (2 * mu * mu / m.impratio) : tran;
      }
      const float ps = pos[r0], mg = marg[r0];
      const float imp = impedance(si, ps, mg);
      float R = (1 - imp) * diag / imp;
      R = R > kMinVal ? R : kMinVal;
      const float dmax = clampf(si[1], 0.0001f, 0.9999f);
      float K, B;
      if (sr[0] > 0) {
        float tc = sr[0], dr = sr[1];
        if (!(m.disableflags & MRS_DSBL_REFSAFE) && tc < 2 * m.timestep) tc = 2 * m.timestep;
        K = 1 / (dmax * dmax * tc * tc * dr * dr);
        B = 2 / (dmax * tc);
      } else {
        K = -sr[0] / (dmax * dmax);
        B = -sr[1] / dmax;
      }
      const float pterm = t == EFC_FRICTION ? 0.0f : K * imp * (ps - mg);
      const float jval = t == EFC_FRICTION ? 1.0f : (t == EFC_LIMIT ? floss[r0] : 0.0f);
      Hdr h{};
      h.a = (v4f){__int_as_float(r0), __int_as_float(code),
                  __int_as_float((t1 + 1) | ((t2 + 1) << 8) | (nr << 16) | (dim << 20) | ((t1 < 0 ? 0xff : il) << 24)), mu};
      h.b = (v4f){R, B, pterm, bound};
      // what the records phase reads per item: the contact's position, bodies, frame and roots (no
      // dependent chain contact -> pair -> geom -> body per item there), or the friction / limit
      // row's J value and dof
      if (t == EFC_CONTACT) {
        const gfloat* crec = scr + S.con + kConRec * id;
        const int p = __float_as_int(crec[0]);
        const int b1 = m.geom_bodyid[m.pair_g1[p]], b2 = m.geom_bodyid[m.pair_g2[p]];
        h.c = (v4f){crec[2], crec[3], crec[4], __int_as_float(b1 | (b2 << 16))};
        h.d = (v4f){crec[5], crec[6], crec[7], crec[8]};
        h.e = (v4f){crec[9], crec[10], crec[11], crec[12]};
        h.f = (v4f){crec[13], __int_as_float(m.body_rootid[b1] | (m.body_rootid[b2] << 16)), 0.0f, 0.0f};
      } else {
        h.c = (v4f){jval, 0.0f, 0.0f, __int_as_float(t == EFC_FRICTION ? id : m.jnt_dofadr[id])};
      }
      h.f.z = __int_as_float(q0);
      if (hreg) {
        hv = h;
      } else {
        __attribute__((address_space(1))) v4f* o = (__attribute__((address_space(1))) v4f*)(hdr + kHdr * q0);
        o[0] = h.a; o[1] = h.b; o[2] = h.c; o[3] = h.d; o[4] = h.e; o[5] = h.f;
      }
    }
  }
  wsync();
  SUB_ADD(PH_CON_ROWS, t_sub);
  t_sub = SUB_T();

  // --- 3. records, one item per pipe per level: J of the item's rows from the contact Jacobian
  // (jc: normal and two tangent rows, pyramid edges jc0 +- mu jck), Y = L^-1 J' of the three jc
  // vectors in one interleaved forward substitution, impedance once per item; the row scalars that
  // need J itself (J qvel, J qacc_smooth, J qacc_warmstart) are taken here, so records hold Y only
  gfloat* quadtab = scr + S.efc_quad;  // per pipe, its first 16 items in order: record | rows << 16
  int my_nq = 0;                        // items of this lane's pipe
  // Y through the inverse factor when the layout holds one and every tree fits the 8-term product
  const bool use_linv = L.Li != 0 && m.tree_nmax <= 8 && !(m.sparse_off & 8);
  if (use_linv) tree_linv(m, s, L, lane);
  const bool warm = !(m.disableflags & MRS_DSBL_WARMSTART);
  {
    const int my_end = my_start + my_n;
    int qc = my_start;
    // hreg: the pipe's next item is the lowest lane left in its pending mask (scalar find-first),
    // its header is fetched from that lane by permute; otherwise headers are read from the scratch
    // one item ahead (loads in flight while the current item is built)
    auto load_hdr = [&](int q) {
      const gfloat* h = hdr + kHdr * q;
      Hdr o;
      o.a = *(const __attribute__((address_space(1))) v4f*)h;
      o.b = *(const __attribute__((address_space(1))) v4f*)(h + 4);
      o.c = *(const __attribute__((address_space(1))) v4f*)(h + 8);
      o.d = *(const __attribute__((address_space(1))) v4f*)(h + 12);
      o.e = *(const __attribute__((address_space(1))) v4f*)(h + 16);
      o.f = *(const __attribute__((address_space(1))) v4f*)(h + 20);
      return o;
    };
    auto perm4 = [](v4f v, int src) {
      return (v4f){__shfl(v.x, src), __shfl(v.y, src), __shfl(v.z, src), __shfl(v.w, src)};
    };
    Hdr nxt{};
    if (!hreg) nxt = load_hdr(qc < my_end ? qc : 0);
    unsigned long long t_rj = 0, t_rs = 0, t_rr = 0;  // timing build: records sub-phases
    (void)t_rj; (void)t_rs; (void)t_rr;
    #pragma unroll 1
    for (;;) {
      unsigned long long t_it = SUB_T();
      Hdr cur;
      bool act;
      if (hreg) {
        int src = 0;
        act = false;
        unroll<NP>([&](auto pc) {
          constexpr int q = decltype(pc)::value;
          const unsigned long long pm = pend[q];
          const int lq = pm ? __builtin_ctzll(pm) : 0;
          if (pipe == q) { src = lq; act = pm != 0; }
          pend[q] = pm & (pm - 1);
        });
        if (!__any(act)) break;
        cur.a = perm4(hv.a, src); cur.b = perm4(hv.b, src); cur.c = perm4(hv.c, src);
        cur.d = perm4(hv.d, src); cur.e = perm4(hv.e, src); cur.f = perm4(hv.f, src);
      } else {
        act = qc < my_end;
        if (!__any(act)) break;
        cur = nxt;
        const int nr_ = (__float_as_int(cur.a.z) >> 16) & 0xf;
        const int qn = qc + (act ? nr_ : 0);
        nxt = load_hdr(qn < my_end ? qn : 0);
      }
      const int q0 = act ? (hreg ? __float_as_int(cur.f.z) : qc) : 0;  // record 0 always starts an item
      const v4f h0 = cur.a, h1 = cur.b, h2 = cur.c, h3 = cur.d, h4 = cur.e;
      const float h20 = cur.f.x;
      const int roots = __float_as_int(cur.f.y);
      const int r0 = __float_as_int(h0.x), code = __float_as_int(h0.y), pk = __float_as_int(h0.z);
      const float mu = h0.w, R = h1.x, B = h1.y, pterm = h1.z, bound = h1.w;
      const int t = code >> 16, id = code & 0xffff;
      const int t1 = (pk & 0xff) - 1, t2 = ((pk >> 8) & 0xff) - 1, nr = (pk >> 16) & 0xf, dim = (pk >> 20) & 0xf;
      const int isl = (pk >> 24) & 0xff;
      const unsigned ip = static_cast<unsigned>(__shfl(static_cast<int>(ipack), isl == 0xff ? 0 : isl));
      const SlotMap sm = isl_ok ? (isl == 0xff ? SlotMap{-1, 0, 0, 0, 0} : island_slot_map(s, L, ip, slot))
                                : slot_map(s, L, t1, t2, slot);
      const int d = sm.d;
      float jc[3] = {0, 0, 0};
      if (t == EFC_CONTACT) {
        if (d >= 0) {
          const int bb = __float_as_int(h2.w);
          const int b1 = bb & 0xffff, b2 = bb >> 16;
          const float cp[3] = {h2.x, h2.y, h2.z};
          const float fr[9] = {h3.x, h3.y, h3.z, h3.w, h4.x, h4.y, h4.z, h4.w, h20};
          float c1[3], c2[3];
          jac_col_blk(s, L, b1, roots & 0xffff, cp, d, c1);
          jac_col_blk(s, L, b2, roots >> 16, cp, d, c2);
          const float dc[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
          for (int i = 0; i < 3; ++i) jc[i] = fr[3 * i] * dc[0] + fr[3 * i + 1] * dc[1] + fr[3 * i + 2] * dc[2];
        }
      } else {
        // friction loss: e_dof; limit: +-e_dof (dof and J value in the header)
        jc[0] = d == __float_as_int(h2.w) ? h2.x : 0.0f;
      }
      float yc[3];
#ifdef MRS_PHASE_TIMING
      { const unsigned long long t_ = SUB_T(); t_rj += t_ - t_it; t_it = t_; }
#endif
      if (use_linv) pipe_linv3(s + L.Li, sm, pbase, jc, yc);
      else pipe_lsolve3(m, s + L.L, sm, pbase, jc, yc);
#ifdef MRS_PHASE_TIMING
      { const unsigned long long t_ = SUB_T(); t_rs += t_ - t_it; t_it = t_; }
#endif
      const float qv = d >= 0 ? s[L.qvel + d] : 0.0f, qs = d >= 0 ? s[L.qacc_smooth + d] : 0.0f;
      const float qw = warm && d >= 0 ? s[L.qacc_ws + d] : 0.0f;
      if (act && slot == 0 && my_nq < 16) quadtab[pipe * 16 + my_nq] = __int_as_float(q0 | (nr << 16));
      float Yk[3] = {0, 0, 0};  // Y of the item's earlier rows (for the couplings)
      unroll<4>([&](auto jcst) {
        constexpr int j = decltype(jcst)::value;
        constexpr int k = 1 + (j >> 1);
        constexpr float sg = (j & 1) ? -1.0f : 1.0f;
        const float J = dim == 1 ? jc[0] : jc[0] + sg * mu * jc[k];
        const float Y = dim == 1 ? yc[0] : yc[0] + sg * mu * yc[k];
        if (j == 0 || __any(act && j < nr)) {
          const float vel = gsum<P>(J * qv), jqs = gsum<P>(J * qs), yy = gsum<P>(Y * Y);
          const float jw = warm ? gsum<P>(J * qw) : 0.0f;
          const float aref = -B * vel - pterm;
          float cpl[3] = {0, 0, 0};
          unroll<3>([&](auto sc) {
            constexpr int s_ = decltype(sc)::value;
            if constexpr (s_ < j) cpl[s_] = gsum<P>(Y * Yk[s_]);
          });
          if constexpr (j < 3) Yk[j] = Y;
          if (act && j < nr) {
            gfloat* o = rec + (q0 + j) * RF;
            o[slot] = Y;
            o[P + slot] = __int_as_float(d);
            if (slot == 0) {
              *(__attribute__((address_space(1))) v4f*)(o + 2 * P) = (v4f){aref, R, yy + R, bound};
              *(__attribute__((address_space(1))) v4f*)(o + 2 * P + 4) = (v4f){jqs - aref, cpl[0], cpl[1], cpl[2]};
              o[2 * P + 8] = jw - aref;
              rowof[q0 + j] = __int_as_float(r0 + j);
            }
          }
        }
      });
      qc += act ? nr : 0;
      my_nq += act ? 1 : 0;
#ifdef MRS_PHASE_TIMING
      t_rr += SUB_T() - t_it;
#endif
    }
#ifdef MRS_PHASE_TIMING
    if (__lane_id() == 0) {
      atomicAdd(&g_phase_cycles[PH_REC_J], t_rj);
      atomicAdd(&g_phase_cycles[PH_REC_SOLVE], t_rs);
      atomicAdd(&g_phase_cycles[PH_REC_ROWS], t_rr);
    }
#endif
  }
  const int nq_max = uniform_int(wave_max(my_nq));
  wsync();
  SUB_ADD(PH_CON_REC, t_sub);
  t_sub = SUB_T();
  // the qacc-tracking solvers below work on w = L' qacc (the dual solve does not read qa)
  const DofTree dtree = dof_tree_lds(m, s, L, lane);
  {
    const float ws = tree_lt_mul(m, dtree, qacc_s);
    if (lane < nv) qa[lane] = ws;
  }

  // --- island-dual register solve (P = 16, island slot frames, at most kDualLevels rows per pipe).
  // mj_solPGS on the dual, as the oracle's fwd_constraint: row r's residual g_r = b_r + sum_s AR_rs f_s
  // is kept, not recomputed from qacc.  Lane (pipe, slot) holds the rows at levels 16 j + slot of its
  // pipe ("held rows") with their Delassus rows AR[j][l] = J_(16j+slot) M^-1 J_l' (+ R on the
  // diagonal) for every level l of the pipe, zero across islands.  A level l is then branch-free and
  // touches no memory: the owner lane's clamped step delta = med3(-g / A, lo - f, hi - f), one DPP row
  // broadcast of it folded into the FMAs g_r += AR_rl delta of every held row (the same Gauss-Seidel
  // iterates as the row-serial sweep), and the owner's share of the sweep improvement -delta (res +
  // A delta / 2) -- no LDS round trip of qacc and no reduction on the chain.  AR is formed once per
  // step from the records: lane slot's held row J (16 slots) times each level's M^-1 J' broadcast slot
  // by slot (DPP row broadcast folded into the FMA).
  if constexpr (P == 16) {
    if (isl_ok && nlev <= kDualLevels && !(m.sparse_off & 1)) {
      constexpr int NL = kDualLevels, NJ = NL / 16;
      const int nch = (nlev + 15) >> 4;  // 16-level chunks of the sweeps (AR zero past nlev)
      typedef float v2f __attribute__((ext_vector_type(2)));
      // ARn[j][l] = -AR_rl / A_rr of held row r = 16 j + slot: the sweeps carry the normalised
      // residual gn_r = -g_r / A_rr (the unclamped step), so a level's step is one med3 of it
      float ARn[NJ][NL];
      float gn[NJ], nia[NJ], A[NJ], bb[NJ], fr[NJ];
      v2f lh[NJ];    // (lo - f, hi - f) of each held row
      int hisl[NJ];  // island tag of each held row: the dof of its slot 0 (-1: none)
      {
        float Jt[NJ][16];
        // held-row scalars and J over its 16 slots from the records (neutral rows past the pipe's
        // own: J = 0, bounds [0, inf))
        unroll<NJ>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const int k = 16 * j + slot;
          const bool act = k < my_n;
          const gfloat* o = rec + (act ? my_start + k : 0) * RF;
          unroll<4>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const v4f v = *(const __attribute__((address_space(1))) v4f*)(o + 4 * q);
            Jt[j][4 * q] = act ? v.x : 0.0f; Jt[j][4 * q + 1] = act ? v.y : 0.0f;
            Jt[j][4 * q + 2] = act ? v.z : 0.0f; Jt[j][4 * q + 3] = act ? v.w : 0.0f;
          });
          const v4f sc = *(const __attribute__((address_space(1))) v4f*)(o + 2 * P);
          const float bound = sc.w;
          lh[j] = (v2f){act && bound >= 0 ? -bound : 0.0f,     // friction loss: [-frictionloss, frictionloss]
                        act && bound >= 0 ? bound : 3.0e38f};  // others: [0, inf)
          bb[j] = act ? o[2 * P + 4] : 0.0f;
          fr[j] = act ? sc.y : 0.0f;                           // R, folded into the diagonal below
          hisl[j] = act ? __float_as_int(o[P]) : -1;
        });
        // AR[j][l] = Y_(16j+slot) . Y_l.  Level l's Y is already in registers: it is held row l / 16
        // of lane l % 16 (Jt, zero past the pipe's rows), so slot q of it is one DPP row broadcast of
        // Jt[l / 16][q] from that lane, folded into the FMAs of the three held rows -- the records are
        // read once here, not again per level
        unroll<NL>([&](auto lc) {
          constexpr int l = decltype(lc)::value;
          unroll<NJ>([&](auto jc) { ARn[decltype(jc)::value][l] = 0.0f; });
          if (l < nlev) {
            const int il = __float_as_int(rowb<l % 16>(__int_as_float(hisl[l / 16])));
            unroll<NJ>([&](auto jc) {
              constexpr int j = decltype(jc)::value;
              float a0 = 0, a1 = 0;
              unroll<16>([&](auto sc) {
                constexpr int q = decltype(sc)::value;
                if constexpr (q & 1) a1 += Jt[j][q] * rowb<l % 16>(Jt[l / 16][q]);
                else a0 += Jt[j][q] * rowb<l % 16>(Jt[l / 16][q]);
              });
              float a = a0 + a1;
              const bool diag = l / 16 == j && slot == l % 16;
              if (diag) a += fr[j];  // + R_rr
              ARn[j][l] = (hisl[j] == il && hisl[j] >= 0) || diag ? a : 0.0f;
            });
          }
        });
      }
      // A_rr from AR itself (the step and the residual update use the same value, as the oracle's AR),
      // then the rows normalised by -1 / A_rr
      unroll<NJ>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        float a = 0;
        unroll<16>([&](auto oc) {
          constexpr int o = decltype(oc)::value;
          if constexpr (16 * j + o < NL) a = slot == o ? ARn[j][16 * j + o] : a;
        });
        a = 16 * j + slot < my_n ? a : 1.0f;
        A[j] = a;
        nia[j] = -1.0f / a;
        unroll<NL>([&](auto lc) { ARn[j][decltype(lc)::value] *= nia[j]; });
      });
      SUB_ADD(PH_CON_DEL, t_sub);
      t_sub = SUB_T();
      // warm start: forces of mj_constraintUpdate at qacc_warmstart (J qacc_warmstart - aref from
      // the record), kept if the dual cost is negative
      unroll<NJ>([&](auto jc) { fr[decltype(jc)::value] = 0.0f; });
      if (warm) {
        unroll<NJ>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const int k = 16 * j + slot;
          const bool act = k < my_n;
          const gfloat* o = rec + (act ? my_start + k : 0) * RF;
          const float jar = act ? o[2 * P + 8] : 0.0f;
          if (act) {
            const float R = o[2 * P + 1];
            const float D = 1.0f / R, hi = lh[j].y;
            fr[j] = lh[j].x < 0 ? (jar <= -R * hi ? hi : (jar >= R * hi ? -hi : -D * jar))
                                : (jar < 0 ? -D * jar : 0.0f);
          }
        });
      }
      // normalised residuals gn = -(b + AR f) / A; warm start kept if the dual cost
      // f' (AR f / 2 + b) = f' (g + b) / 2 is negative
      unroll<NJ>([&](auto jc) { gn[decltype(jc)::value] = nia[decltype(jc)::value] * bb[decltype(jc)::value]; });
      if (warm) {
        unroll<NL>([&](auto lc) {
          constexpr int l = decltype(lc)::value;
          if (l < nlev) {
            const float fl = rowb<l % 16>(fr[l / 16]);
            unroll<NJ>([&](auto jc) { gn[decltype(jc)::value] += ARn[decltype(jc)::value][l] * fl; });
          }
        });
        float c = 0;
        unroll<NJ>([&](auto jc) { constexpr int j = decltype(jc)::value; c += fr[j] * (bb[j] - A[j] * gn[j]); });
        if (gsum<64>(c) > 0) {
          unroll<NJ>([&](auto jc) { constexpr int j = decltype(jc)::value; fr[j] = 0.0f; gn[j] = nia[j] * bb[j]; });
        }
      }
      unroll<NJ>([&](auto jc) { constexpr int j = decltype(jc)::value; lh[j] -= (v2f){fr[j], fr[j]}; });
      SUB_ADD(PH_CON_WARM, t_sub);
      t_sub = SUB_T();
      // sweeps: level k's owner (slot k % 16, held row k / 16) takes the clamped step, every held row
      // of the pipe moves its normalised residual by ARn delta (DPP row broadcast of the step folded
      // into the FMA); the owner's improvement term -delta (res + A delta / 2) = A delta (gn - delta/2)
      // is accumulated per held row and scaled by A once per sweep
      // A held row moves its own bounds and improvement term only at its own level, and reads them
      // nowhere else in the sweep, so the owner just keeps its residual at that level (gb, one lane
      // select with a constant lane mask) and the bounds / improvement of all held rows are updated
      // together after the sweep: a level is med3 + DPP broadcast + the FMAs + one select.  Levels run
      // in chunks of 16 (levels past nlev hold neutral rows: zero AR rows, step 0).
      int nit = 0;
      #pragma unroll 1
      for (int it = 0; it < m.iterations; ++it) {
        float gb[NJ];
        unroll<NJ>([&](auto jc) { gb[decltype(jc)::value] = gn[decltype(jc)::value]; });
        unroll<NJ>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          if (j < nch) {
            unroll<16>([&](auto oc) {
              constexpr int o = decltype(oc)::value, k = 16 * j + o;
              const float cand = __builtin_amdgcn_fmed3f(gn[j], lh[j].x, lh[j].y);
              gb[j] = sel_slot16<o>(gn[j], gb[j]);
              // the chain to the next level's step runs through held block j only: its update takes
              // the broadcast as the FMA's DPP operand (med3 -> fmac_dpp -> med3); the other blocks
              // use a separate broadcast off that chain
              if constexpr (NJ == 3) {
                constexpr int ja = (j + 1) % 3, jb = (j + 2) % 3;
                fmac3_rowb<o>(gn[j], gn[ja], gn[jb], cand, ARn[j][k], ARn[ja][k], ARn[jb][k]);
              } else {
                gn[j] = fmac_rowb<o>(gn[j], ARn[j][k], cand);
                const float dl = rowb<o>(cand);
                unroll<NJ>([&](auto jc2) {
                  constexpr int j2 = decltype(jc2)::value;
                  if constexpr (j2 != j) gn[j2] += ARn[j2][k] * dl;
                });
              }
            });
          }
        });
        float imp = 0;
        unroll<NJ>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          const float dm = __builtin_amdgcn_fmed3f(gb[j], lh[j].x, lh[j].y);
          imp += A[j] * fmaf(dm, fmaf(-0.5f, dm, gb[j]), 0.0f);
          lh[j] -= (v2f){dm, dm};
        });
        const float improvement = gsum<64>(imp);
        nit = it + 1;
        if (improvement * m.pgs_scale < m.tolerance) break;
      }
      if (lane == 0) s[L.niter] = __int_as_float(nit);
      SUB_ADD(PH_CON_PGS, t_sub);
      // forces f = lo - (lo - f); z = sum Y' f per level, then qfrc_constraint and qacc from z
      unroll<NJ>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const int k = 16 * j + slot;
        const float bound = k < my_n ? rec[(my_start + k) * RF + 2 * P + 3] : -1.0f;
        fr[j] = (bound >= 0 ? -bound : 0.0f) - lh[j].x;
      });
      if (lane < nv) tmp[lane] = 0;
      wsync();
      // 16 levels at a time: every record load of the chunk is in flight together (one vmcnt wait per
      // chunk, not one per level), the level's force comes from its owner slot by a DPP row broadcast,
      // and the per-dof sums accumulate in level order (a dof belongs to one island, so one pipe and
      // one slot write it: no two lanes of an instruction share an address)
      unroll<NJ>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if (j < nch) {
          float Yl[16];
          int dl[16];
          unroll<16>([&](auto oc) {
            constexpr int o = decltype(oc)::value;
            const int l = 16 * j + o;
            const gfloat* r = rec + (l < my_n ? my_start + l : 0) * RF;
            Yl[o] = r[slot];
            dl[o] = l < my_n ? __float_as_int(r[P + slot]) : -1;
          });
          unroll<16>([&](auto oc) {
            constexpr int o = decltype(oc)::value;
            const float f = rowb<o>(fr[j]);
            if (dl[o] >= 0) tmp[dl[o]] += Yl[o] * f;
          });
        }
      });
      unroll<NJ>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const int k = 16 * j + slot;
        if (k < my_n) ffg[__float_as_int(rowof[my_start + k])] = fr[j];
      });
      wsync();
      return tree_epilogue(m, s, L, tmp, qa, qacc_s, lane);
    }
  }

  // --- item-blocked register solve: P = 16 and at most kRegQuads items per pipe.  Item i of a pipe
  // takes levels 4i..4i+3 (its 1 or 4 rows, the rest neutral: J = 0, R = a = 1, bounds [0, inf)), and
  // all of an item's rows share one dof per slot (a contact's rows span the same two trees).  A sweep
  // visits an item with one LDS read of qacc, the four J qacc sums as independent DPP reductions, the
  // rows' Gauss-Seidel updates as a scalar chain through the couplings c_rs = J_r M^-1 J_s' (row r
  // sees qacc + sum_{s<r} M^-1 J_s' df_s, so J_r qacc moves by sum c_rs df_s: the same iterates as
  // the row-serial sweep), and one LDS write of qacc + sum_r M^-1 J_r' df_r -- all in w = L' qacc,
  // where J qacc = Y . w and a step moves w by Y df.  Lane (pipe, slot) keeps Y of its slot for every
  // level; the scalars of level k live in slot k % 16.
  if constexpr (P == 16) {
    if (nq_max <= kRegQuads && !(m.sparse_off & 2)) {
      constexpr int NQ = kRegQuads, NL = 4 * NQ, NB = NL / 16;
      float Yr[NL], sa[NB], sR[NB], sA[NB], sLo[NB], sHi[NB], sB[NB], sW[NB], fr[NB];
      float sC0[NB], sC1[NB], sC2[NB];
      unsigned dpk[(NQ + 3) / 4];
      const unsigned dummy = static_cast<unsigned>(nv);
      if (lane == 0) { qa[nv] = 0; tmp[nv] = 0; }
      unroll<(NQ + 3) / 4>([&](auto ic) { dpk[decltype(ic)::value] = dummy * 0x01010101u; });
      unroll<NB>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        sa[i] = 0; sR[i] = 1; sA[i] = 1; sLo[i] = 0; sHi[i] = 3.0e38f; sB[i] = 0; sW[i] = 0; fr[i] = 0;
        sC0[i] = 0; sC1[i] = 0; sC2[i] = 0;
      });
      unroll<NQ>([&](auto qc) {
        constexpr int i = decltype(qc)::value;
        unroll<4>([&](auto rc) { Yr[4 * i + decltype(rc)::value] = 0; });
        if (i < nq_max) {
          const bool act = i < my_nq;
          const int qt = act ? __float_as_int(quadtab[pipe * 16 + i]) : 0;
          const int q = qt & 0xffff, nr = qt >> 16;
          const int d = __float_as_int(rec[q * RF + P + slot]);
          if (act) {
            const unsigned di = d >= 0 ? static_cast<unsigned>(d) : dummy;
            dpk[i / 4] = (dpk[i / 4] & ~(0xffu << (8 * (i % 4)))) | (di << (8 * (i % 4)));
          }
          unroll<4>([&](auto rc) {
            constexpr int r = decltype(rc)::value, k = 4 * i + r;
            if (act && r < nr) {
              const gfloat* o = rec + (q + r) * RF;
              Yr[k] = o[slot];
              if (slot == k % 16) {
                const v4f sc = *(const __attribute__((address_space(1))) v4f*)(o + 2 * P);
                const v4f sd = *(const __attribute__((address_space(1))) v4f*)(o + 2 * P + 4);
                sa[k / 16] = sc.x; sR[k / 16] = sc.y; sA[k / 16] = sc.z;
                sLo[k / 16] = sc.w >= 0 ? -sc.w : 0.0f;     // friction: [-frictionloss, frictionloss]
                sHi[k / 16] = sc.w >= 0 ? sc.w : 3.0e38f;   // others: [0, inf)
                sB[k / 16] = sd.x;
                sC0[k / 16] = sd.y; sC1[k / 16] = sd.z; sC2[k / 16] = sd.w;
                sW[k / 16] = o[2 * P + 8];
              }
            }
          });
        }
      });
      wsync();
      auto dof_of = [&](auto qc) {
        constexpr int i = decltype(qc)::value;
        return static_cast<int>(__builtin_amdgcn_ubfe(dpk[i / 4], 8 * (i % 4), 8));
      };
      // warm start
      unroll<NQ>([&](auto qc) {
        constexpr int i = decltype(qc)::value;
        if (i < nq_max) {
          unroll<4>([&](auto rc) {
            constexpr int k = 4 * i + decltype(rc)::value;
            float f = 0;
            if (warm) {
              const float R = rowb<k % 16>(sR[k / 16]);
              const float lo = rowb<k % 16>(sLo[k / 16]), hi = rowb<k % 16>(sHi[k / 16]);
              const float jar = rowb<k % 16>(sW[k / 16]);
              const float D = 1.0f / R;
              if (lo < 0) f = jar <= -R * hi ? hi : (jar >= R * hi ? -hi : -D * jar);
              else f = jar < 0 ? -D * jar : 0.0f;
            }
            if (slot == k % 16) fr[k / 16] = f;  // neutral rows: J = 0, aref = 0 -> f = 0
          });
        }
      });
      if (warm) {
        if (lane < nv) tmp[lane] = 0;
        wsync();
        unroll<NQ>([&](auto qc) {
          constexpr int i = decltype(qc)::value;
          if (i < nq_max) {
            const int d = dof_of(qc);
            float acc = 0;
            unroll<4>([&](auto rc) {
              constexpr int k = 4 * i + decltype(rc)::value;
              acc += Yr[k] * rowb<k % 16>(fr[k / 16]);
            });
            tmp[d] += acc;
          }
        });
        wsync();
        float cost = 0;
        unroll<NQ>([&](auto qc) {
          constexpr int i = decltype(qc)::value;
          if (i < nq_max) {
            const float t = tmp[dof_of(qc)];
            unroll<4>([&](auto rc) {
              constexpr int k = 4 * i + decltype(rc)::value;
              const float jv = gsum<16>(Yr[k] * t);
              const float f = rowb<k % 16>(fr[k / 16]), R = rowb<k % 16>(sR[k / 16]), b = rowb<k % 16>(sB[k / 16]);
              cost += f * (0.5f * (jv + R * f) + b);
            });
          }
        });
        cost = gsum<64>(slot == 0 ? cost : 0.0f);
        if (cost > 0) {
          unroll<NB>([&](auto ic) { fr[decltype(ic)::value] = 0; });
        } else if (lane < nv) {
          qa[lane] += tmp[lane];
        }
        wsync();
      }
      SUB_ADD(PH_CON_WARM, t_sub);
      t_sub = SUB_T();
      // PGS sweeps, one item at a time
      int slot_v = slot;
      int nit = 0;
      #pragma unroll 1
      for (int it = 0; it < m.iterations; ++it) {
#pragma unroll
        for (int i = 0; i < (NQ + 3) / 4; ++i) asm volatile("" : "+v"(dpk[i]));
        asm volatile("" : "+v"(slot_v));
        float improvement = 0;
        unroll<NQ>([&](auto qc) {
          constexpr int i = decltype(qc)::value;
          if (i < nq_max) {
            const int d = dof_of(qc);
            const float qd = qa[d];
            float jq[4], df[4] = {0, 0, 0, 0};
            unroll<4>([&](auto rc) {
              constexpr int r = decltype(rc)::value;
              jq[r] = gsum<16>(Yr[4 * i + r] * qd);
            });
            float upd = 0;
            unroll<4>([&](auto rc) {
              constexpr int r = decltype(rc)::value, k = 4 * i + r;
              float c = jq[r];
              if constexpr (r > 0) c += rowb<k % 16>(sC0[k / 16]) * df[0];
              if constexpr (r > 1) c += rowb<k % 16>(sC1[k / 16]) * df[1];
              if constexpr (r > 2) c += rowb<k % 16>(sC2[k / 16]) * df[2];
              const float f0 = rowb<k % 16>(fr[k / 16]);
              const float aref = rowb<k % 16>(sa[k / 16]), R = rowb<k % 16>(sR[k / 16]);
              const float a = rowb<k % 16>(sA[k / 16]);
              const float lo = rowb<k % 16>(sLo[k / 16]), hi = rowb<k % 16>(sHi[k / 16]);
              const float res = c - aref + R * f0;
              const float nf = __builtin_amdgcn_fmed3f(f0 - res * __builtin_amdgcn_rcpf(a), lo, hi);
              df[r] = nf - f0;
              upd += Yr[k] * df[r];
              fr[k / 16] = slot_v == k % 16 ? nf : fr[k / 16];
              improvement -= df[r] * res + 0.5f * df[r] * df[r] * a;
            });
            qa[d] = qd + upd;
          }
        });
        improvement = gsum<64>(slot_v == 0 ? improvement : 0.0f);
        nit = it + 1;
        if (improvement * m.pgs_scale < m.tolerance) break;
      }
      if (lane == 0) s[L.niter] = __int_as_float(nit);
      wsync();
      SUB_ADD(PH_CON_PGS, t_sub);
      // qfrc_constraint = J' f and the forces out (by row index, for mj_rnePostConstraint)
      if (lane < nv) tmp[lane] = 0;
      wsync();
      unroll<NQ>([&](auto qc) {
        constexpr int i = decltype(qc)::value;
        if (i < nq_max) {
          float acc = 0;
          unroll<4>([&](auto rc) {
            constexpr int k = 4 * i + decltype(rc)::value;
            acc += Yr[k] * rowb<k % 16>(fr[k / 16]);
          });
          tmp[dof_of(qc)] += acc;
        }
      });
      unroll<NB>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        const int i = 4 * b + slot / 4, r = slot % 4;  // level 16 b + slot = item i, row r
        if (i < my_nq && i < NQ) {
          const int qt = __float_as_int(quadtab[pipe * 16 + i]);
          if (r < (qt >> 16)) ffg[__float_as_int(rowof[(qt & 0xffff) + r])] = fr[b];
        }
      });
      wsync();
      return tree_epilogue(m, s, L, tmp, qa, qacc_s, lane);
    }
  }

  // --- register-resident solve: P = 16 and at most kRegLevels rows per pipe, on w = L' qacc.  Lane
  // (pipe, slot) keeps Y and the dof of its slot for every level (slots outside the row's trees point
  // at a dummy LDS word after qacc, with Y = 0); the row scalars and the force of level k live
  // in slot k % 16 and reach the pipe by one DPP row broadcast each.  A level is branch-free: pipes
  // with fewer rows run neutral rows (J = 0, R = a = 1, bounds [0, inf)), whose force stays 0.
  // Sweeps touch LDS only for qacc.
  if constexpr (P == 16) {
    if (nlev <= kRegLevels && !(m.sparse_off & 4)) {
      constexpr int NL = kRegLevels, NB = NL / 16;
      float Yr[NL], sa[NB], sR[NB], sA[NB], sLo[NB], sHi[NB], sW[NB], fr[NB];
      unsigned dpk[NL / 4];
      const unsigned dummy = static_cast<unsigned>(nv);
      if (lane == 0) { qa[nv] = 0; tmp[nv] = 0; }
      unroll<NL / 4>([&](auto ic) { dpk[decltype(ic)::value] = dummy * 0x01010101u; });
      unroll<NB>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        sa[i] = 0; sR[i] = 1; sA[i] = 1; sLo[i] = 0; sHi[i] = 3.0e38f; sW[i] = 0; fr[i] = 0;
      });
      unroll<NL>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        Yr[k] = 0;
        if (k < nlev) {
          const bool act = k < my_n;
          const gfloat* o = rec + (act ? my_start + k : 0) * RF;
          const int d = __float_as_int(o[P + slot]);
          if (act) {
            Yr[k] = o[slot];
            const unsigned di = d >= 0 ? static_cast<unsigned>(d) : dummy;
            dpk[k / 4] = (dpk[k / 4] & ~(0xffu << (8 * (k % 4)))) | (di << (8 * (k % 4)));
          }
          if (act && slot == k % 16) {
            const v4f sc = *(const __attribute__((address_space(1))) v4f*)(o + 2 * P);
            sa[k / 16] = sc.x; sR[k / 16] = sc.y; sA[k / 16] = sc.z;
            sLo[k / 16] = sc.w >= 0 ? -sc.w : 0.0f;     // friction: [-frictionloss, frictionloss]
            sHi[k / 16] = sc.w >= 0 ? sc.w : 3.0e38f;   // others: [0, inf)
            sW[k / 16] = o[2 * P + 8];
          }
        }
      });
      wsync();
      auto dof_of = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        return static_cast<int>(__builtin_amdgcn_ubfe(dpk[k / 4], 8 * (k % 4), 8));
      };
      // warm start
      unroll<NL>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k < nlev) {
          float f = 0;
          if (warm) {
            const float R = rowb<k % 16>(sR[k / 16]);
            const float lo = rowb<k % 16>(sLo[k / 16]), hi = rowb<k % 16>(sHi[k / 16]);
            const float jar = rowb<k % 16>(sW[k / 16]);
            const float D = 1.0f / R;
            if (lo < 0) f = jar <= -R * hi ? hi : (jar >= R * hi ? -hi : -D * jar);
            else f = jar < 0 ? -D * jar : 0.0f;
          }
          if (slot == k % 16 && k < my_n) fr[k / 16] = f;
        }
      });
      if (warm) {
        if (lane < nv) tmp[lane] = 0;
        wsync();
        unroll<NL>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          if (k < nlev) {
            const int d = dof_of(kc);
            tmp[d] += Yr[k] * rowb<k % 16>(fr[k / 16]);
          }
        });
        wsync();
        float cost = 0;
        unroll<NL>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          if (k < nlev) {
            const int d = dof_of(kc);
            const float jv = gsum<16>(Yr[k] * tmp[d]);
            const float f = rowb<k % 16>(fr[k / 16]), R = rowb<k % 16>(sR[k / 16]);
            const float b = rec[(k < my_n ? my_start + k : 0) * RF + 2 * P + 4];
            if (k < my_n) cost += f * (0.5f * (jv + R * f) + b);
          }
        });
        cost = gsum<64>(slot == 0 ? cost : 0.0f);
        if (cost > 0) {
          unroll<NB>([&](auto ic) { fr[decltype(ic)::value] = 0; });
        } else if (lane < nv) {
          qa[lane] += tmp[lane];
        }
        wsync();
      }
      SUB_ADD(PH_CON_WARM, t_sub);
      t_sub = SUB_T();
      // PGS sweeps
      int slot_v = slot;
      int nit = 0;  // sweeps done (mjData.solver_niter)
      #pragma unroll 1
      for (int it = 0; it < m.iterations; ++it) {
        // opaque per sweep: keeps the per-level dof indices and lane masks from being hoisted out
        // of the sweep loop (they would not fit the register budget next to J and M^-1 J')
#pragma unroll
        for (int i = 0; i < NL / 4; ++i) asm volatile("" : "+v"(dpk[i]));
        asm volatile("" : "+v"(slot_v));
        float improvement = 0;
        unroll<NL>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          if (k < nlev) {
            const int d = dof_of(kc);
            const float qd = qa[d];
            const float f0 = rowb<k % 16>(fr[k / 16]);
            const float aref = rowb<k % 16>(sa[k / 16]), R = rowb<k % 16>(sR[k / 16]);
            const float a = rowb<k % 16>(sA[k / 16]);
            const float lo = rowb<k % 16>(sLo[k / 16]), hi = rowb<k % 16>(sHi[k / 16]);
            const float jq = gsum<16>(Yr[k] * qd);
            const float res = jq - aref + R * f0;
            const float nf = __builtin_amdgcn_fmed3f(f0 - res * __builtin_amdgcn_rcpf(a), lo, hi);
            const float delta = nf - f0;
            qa[d] = qd + Yr[k] * delta;
            fr[k / 16] = slot_v == k % 16 ? nf : fr[k / 16];
            improvement -= delta * res + 0.5f * delta * delta * a;
          }
        });
        improvement = gsum<64>(slot_v == 0 ? improvement : 0.0f);
        nit = it + 1;
        if (improvement * m.pgs_scale < m.tolerance) break;
      }
      if (lane == 0) s[L.niter] = __int_as_float(nit);
      wsync();
      SUB_ADD(PH_CON_PGS, t_sub);
      // qfrc_constraint = J' f and the forces out (by row index, for mj_rnePostConstraint)
      if (lane < nv) tmp[lane] = 0;
      wsync();
      unroll<NL>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k < nlev) {
          const int d = dof_of(kc);
          tmp[d] += Yr[k] * rowb<k % 16>(fr[k / 16]);
        }
      });
      unroll<NB>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const int k = i * 16 + slot;
        if (k < my_n) ffg[__float_as_int(rowof[my_start + k])] = fr[i];
      });
      wsync();
      return tree_epilogue(m, s, L, tmp, qa, qacc_s, lane);
    }
  }

  // --- 4. warm start: forces of mj_constraintUpdate at qacc_warmstart, kept if the dual cost < 0
  #pragma unroll 1
  for (int k = 0; k < nlev; ++k) {
    const bool act = k < my_n;
    const int q = act ? my_start + k : 0;
    const RowRec<P> w = load_rec<P>(rec, q, slot);
    float f = 0;
    if (warm) {
      const float jar = rec[q * RF + 2 * P + 8];
      const float D = 1.0f / w.R;
      if (w.bound >= 0) f = jar <= -w.R * w.bound ? w.bound : (jar >= w.R * w.bound ? -w.bound : -D * jar);
      else f = jar < 0 ? -D * jar : 0.0f;
    }
    if (act && slot == 0) fl[q] = f;
  }
  wsync();
  if (warm) {
    if (lane < nv) tmp[lane] = 0;
    wsync();
    #pragma unroll 1
    for (int k = 0; k < nlev; ++k) {
      const bool act = k < my_n;
      const int q = act ? my_start + k : 0;
      const RowRec<P> w = load_rec<P>(rec, q, slot);
      if (act && w.d >= 0) tmp[w.d] += w.Y * fl[q];
    }
    wsync();
    float cost = 0;
    #pragma unroll 1
    for (int k = 0; k < nlev; ++k) {
      const bool act = k < my_n;
      const int q = act ? my_start + k : 0;
      const RowRec<P> w = load_rec<P>(rec, q, slot);
      const float jv = gsum<P>(act && w.d >= 0 ? w.Y * tmp[w.d] : 0.0f);
      const float f = fl[q];
      const float b = rec[q * RF + 2 * P + 4];
      if (act && slot == 0) cost += f * (0.5f * (jv + w.R * f) + b);
    }
    cost = gsum<64>(cost);
    if (cost > 0) {
      #pragma unroll 1
      for (int q = lane; q < nefc; q += 64) fl[q] = 0;
    } else if (lane < nv) {
      qa[lane] += tmp[lane];
    }
    wsync();
  }

  // --- 5. PGS sweeps: level k = the k-th row of every pipe; next level's record prefetched
  int nit = 0;  // sweeps done (mjData.solver_niter)
  #pragma unroll 1
  for (int it = 0; it < m.iterations; ++it) {
    float improvement = 0;
    RowRec<P> nxt = load_rec<P>(rec, my_n > 0 ? my_start : 0, slot);
    #pragma unroll 1
    for (int k = 0; k < nlev; ++k) {
      const RowRec<P> w = nxt;
      const bool act = k < my_n;
      if (k + 1 < nlev) nxt = load_rec<P>(rec, k + 1 < my_n ? my_start + k + 1 : 0, slot);
      const int q = act ? my_start + k : 0;
      const bool mine = act && w.d >= 0;
      const float qd = mine ? qa[w.d] : 0.0f;
      const float f0 = fl[q];
      const float jq = gsum<P>(mine ? w.Y * qd : 0.0f);
      const float res = jq - w.aref + w.R * f0;
      float nf = f0 - res / w.a;
      if (w.bound >= 0) nf = clampf(nf, -w.bound, w.bound);
      else if (nf < 0) nf = 0;
      const float delta = nf - f0;
      if (mine && delta != 0) qa[w.d] = qd + w.Y * delta;
      if (act && slot == 0) fl[q] = nf;
      if (act) improvement -= delta * res + 0.5f * delta * delta * w.a;
    }
    improvement = gsum<64>(slot == 0 ? improvement : 0.0f);
    wsync();
    nit = it + 1;
    if (improvement * m.pgs_scale < m.tolerance) break;
  }
  if (lane == 0) s[L.niter] = __int_as_float(nit);
  wsync();

  // --- 6. z = sum Y' f (per dof in row order: a dof's rows are in one pipe), then qfrc_constraint
  // and qacc from it; forces out
  if (lane < nv) tmp[lane] = 0;
  wsync();
  #pragma unroll 1
  for (int k = 0; k < nlev; ++k) {
    const bool act = k < my_n;
    const int q = act ? my_start + k : 0;
    const RowRec<P> w = load_rec<P>(rec, q, slot);
    if (act && w.d >= 0) tmp[w.d] += w.Y * fl[q];
  }
  #pragma unroll 1
  for (int q = lane; q < nefc; q += 64) ffg[__float_as_int(rowof[q])] = fl[q];
  wsync();
  return tree_epilogue(m, s, L, tmp, qa, qacc_s, lane);
}

// ---------------------------------------------------------------- primal solvers (Newton, CG)
// mj_solNewton / mj_solCG [upstream engine_solver.c mj_solPrimal]; the algorithm, its stopping rules
// and the restatement choices are stated once in oracle/oracle.c (solve_primal).  Dense rows in the
// env's scratch (J, R, aref, frictionloss); lane j < nv holds dof j of every vector (qacc, M qacc,
// gradient, search direction, M search); row quantities are lane-strided over rows: jar = J qacc -
// aref in efc_b, J search in efc_ARii, the row state in efc_MJ, forces in efc_f.  Newton builds
// H = M + J' diag(D of quadratic rows) J row-per-lane into the LDS factor slot and factors it in
// place (M's factor is not needed again before integrate() refactors); CG preconditions with M's
// factor.  The broadcast buffer for matrix-vector products is L.qacc (written by forward() after).
enum { PST_SAT = 0, PST_QUAD = 1, PST_LINNEG = 2, PST_LINPOS = 3 };
__device__ __forceinline__ int prow_state(bool fric, float R, float fl, float jar) {
  if (fric) {
    const float rf = R * fl;
    return jar <= -rf ? PST_LINNEG : (jar >= rf ? PST_LINPOS : PST_QUAD);
  }
  return jar < 0 ? PST_QUAD : PST_SAT;
}
__device__ __forceinline__ float prow_cost(int st, float R, float fl, float jar) {
  return st == PST_QUAD ? 0.5f * jar * jar / R
                        : (st == PST_LINNEG ? -fl * jar - 0.5f * R * fl * fl
                                            : (st == PST_LINPOS ? fl * jar - 0.5f * R * fl * fl : 0.0f));
}
__device__ __forceinline__ float prow_slope(int st, float R, float fl, float jar) {
  return st == PST_QUAD ? jar / R : (st == PST_LINNEG ? -fl : (st == PST_LINPOS ? fl : 0.0f));
}
// ---- elliptic friction cones (oracle.c ell_block / qcqp2_la / ell_block_min restate them; same
// formulas in fp32).  A contact of condim 3 under cone="elliptic" is a 3-row block (normal, tangent 1,
// tangent 2); its rows carry k + 1 in the efc_floss slot (k = 0, 1, 2; 0 for every other contact row),
// so a block starts where that slot holds 1.
enum { PST_CONE = 4 };
__device__ __forceinline__ bool ell_start(const DevModel& m, const gfloat* type, const gfloat* floss, int r) {
  return m.cone == MRS_CONE_ELLIPTIC && (__float_as_int(type[r]) >> 16) == EFC_CONTACT && floss[r] == 1.0f;
}
// the block's friction coefficient (both tangents: sliding) and regularised cone mu = mu_1 / sqrt(impratio)
__device__ __forceinline__ float ell_friction(const DevModel& m, const gfloat* scr, const gfloat* type, int r) {
  const int c = __float_as_int(type[r]) & 0xffff;
  return m.pair_friction[3 * __float_as_int(scr[m.S.con + kConRec * c])];
}
// zone (PST_SAT top, PST_QUAD bottom, PST_CONE middle) at jar; f, cost and the jar-space Hessian H may
// be null
__device__ __forceinline__ int ell_zone(float ft, float imp, const float D[3], const float jar[3], float* f, float* cost,
                                        float* H) {
  const float mu = ft * rsqrtf(imp);
  const float U[3] = {mu * jar[0], ft * jar[1], ft * jar[2]};
  const float N = U[0], T = sqrtf(U[1] * U[1] + U[2] * U[2]);
  if (N >= mu * T || (T <= 0 && N >= 0)) {
    if (f) { f[0] = f[1] = f[2] = 0; }
    if (cost) *cost = 0;
    if (H) for (int i = 0; i < 9; ++i) H[i] = 0;
    return PST_SAT;
  }
  if (mu * N + T <= 0 || (T <= 0 && N < 0)) {
    float c = 0;
    for (int j = 0; j < 3; ++j) {
      if (f) f[j] = -D[j] * jar[j];
      c += 0.5f * D[j] * jar[j] * jar[j];
    }
    if (cost) *cost = c;
    if (H) for (int i = 0; i < 9; ++i) H[i] = (i % 4 == 0) ? D[i / 4] : 0.0f;
    return PST_QUAD;
  }
  const float Dm = D[0] / (mu * mu * (1 + mu * mu)), NT = N - mu * T;
  if (cost) *cost = 0.5f * Dm * NT * NT;
  if (f) {
    f[0] = -Dm * NT * mu;
    for (int j = 1; j < 3; ++j) f[j] = Dm * NT * mu / T * U[j] * ft;
  }
  if (H) {
    const float S[3] = {mu, ft, ft};
    float HU[9];
    HU[0] = 1;
    for (int j = 1; j < 3; ++j) HU[j] = HU[3 * j] = -mu * U[j] / T;
    for (int j = 1; j < 3; ++j)
      for (int k = 1; k < 3; ++k) HU[3 * j + k] = mu * N / (T * T * T) * U[j] * U[k] + (j == k ? mu * mu - mu * N / T : 0.0f);
    for (int j = 0; j < 3; ++j)
      for (int k = 0; k < 3; ++k) H[3 * j + k] = Dm * S[j] * HU[3 * j + k] * S[k];
  }
  return PST_CONE;
}
// mju_QCQP2 with its multiplier (oracle.c qcqp2_la).  The elliptic PGS block updates below run in
// fp64 (the sweep keeps its iterate in fp64, constraints_dense): the split update converges slowly
// enough that fp32 storage of the block forces alone leaves a noise floor of ~1e-4 in qvel
// (scripts/diag_elliptic_round.py: rounding the oracle's iterate to fp32 moves qvel by 1.2e-4,
// rounding its Delassus rows and b -- the solver's inputs -- by 2e-7), so the iterate, the residuals
// and these updates take the oracle's precision and thresholds
__device__ __forceinline__ double qcqp2_la(double res[2], const double A[4], const double b[2], double d, double r) {
  const double b1 = b[0] * d, b2 = b[1] * d;
  const double A11 = A[0] * d * d, A22 = A[3] * d * d, A12 = A[1] * d * d;
  double la = 0, v1 = 0, v2 = 0;
  #pragma unroll 1
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
  res[0] = v1 * d;
  res[1] = v2 * d;
  return la;
}
// the exact minimiser of 1/2 y'Ay + y'c over |y_t| <= mu y_n (oracle.c ell_block_min): secant /
// bisection on g'(s) = (A y + c)_n - la s with the QCQP inside
__device__ __forceinline__ void ell_block_min(const double A[9], const double c[3], double mu, double y[3]) {
  const double At[4] = {A[4], A[5], A[7], A[8]};
  double x[2];
  double gp_lo = c[0] - mu * sqrt(c[1] * c[1] + c[2] * c[2]), s_lo = 0, gp_hi = 0;
  if (gp_lo >= 0) { y[0] = y[1] = y[2] = 0; return; }
  auto eval = [&](double s) {
    const double bc[2] = {c[1] + A[3] * s, c[2] + A[6] * s};
    const double la = qcqp2_la(x, At, bc, mu, s);
    return A[0] * s + A[1] * x[0] + A[2] * x[1] + c[0] - la * s;
  };
  double s_hi = -c[0] / A[0];
  if (!(s_hi > 0)) s_hi = 1;
  #pragma unroll 1
  for (int k = 0; k < 60; ++k) {
    gp_hi = eval(s_hi);
    if (gp_hi >= 0) break;
    s_lo = s_hi; gp_lo = gp_hi;
    s_hi *= 2;
  }
  #pragma unroll 1
  for (int it = 0; it < 100 && s_hi - s_lo > 1e-14 * (1 + s_hi); ++it) {
    double sn = s_lo - gp_lo * (s_hi - s_lo) / (gp_hi - gp_lo);
    if (!(sn > s_lo + 0.01 * (s_hi - s_lo) && sn < s_hi - 0.01 * (s_hi - s_lo))) sn = 0.5 * (s_lo + s_hi);
    const double gp = eval(sn);
    if (gp == 0) { s_lo = s_hi = sn; break; }
    if (gp < 0) { s_lo = sn; gp_lo = gp; } else { s_hi = sn; gp_hi = gp; }
  }
  const double s = 0.5 * (s_lo + s_hi);
  const double bc[2] = {c[1] + A[3] * s, c[2] + A[6] * s};
  qcqp2_la(x, At, bc, mu, s);
  y[0] = s; y[1] = x[0]; y[2] = x[1];
}

// mj_solPGS's split update of one elliptic block (oracle.c ell_pgs_split): a normal step (old normal
// force 0) or the exact step along the ray of the old force (normal kept >= 0), then the friction by
// mju_QCQP2 with the normal fixed
__device__ __forceinline__ void ell_pgs_split(const double A[9], const double res[3], const double old[3], double mu,
                                              double y[3]) {
  constexpr double kMin = 1e-15;
  y[0] = old[0]; y[1] = old[1]; y[2] = old[2];
  if (A[0] < kMin) return;
  if (old[0] < kMin) {
    y[0] = fmax(old[0] - res[0] / A[0], 0.0);
  } else {
    double Av[3], vAv = 0, vr = 0;
    for (int k = 0; k < 3; ++k) Av[k] = A[3 * k] * old[0] + A[3 * k + 1] * old[1] + A[3 * k + 2] * old[2];
    for (int k = 0; k < 3; ++k) { vAv += old[k] * Av[k]; vr += old[k] * res[k]; }
    if (vAv >= kMin) {
      double x = -vr / vAv;
      if (old[0] + x * old[0] < 0) x = -1.0;
      for (int k = 0; k < 3; ++k) y[k] = old[k] + x * old[k];
    }
  }
  if (y[0] < kMin) { y[0] = fmax(y[0], 0.0); y[1] = y[2] = 0; return; }
  const double At[4] = {A[4], A[5], A[7], A[8]};
  const double dn = y[0] - old[0];
  const double bt[2] = {res[1] + A[3] * dn - (A[4] * old[1] + A[5] * old[2]),
                        res[2] + A[6] * dn - (A[7] * old[1] + A[8] * old[2])};
  double x[2];
  qcqp2_la(x, At, bt, mu, y[0]);
  y[1] = x[0]; y[2] = x[1];
}

// cost change of a row moved from jar j0 (state s0) by dj to state s1, in factored form when the
// state is kept (no cancellation of two nearly equal costs in fp32)
__device__ __forceinline__ float prow_dcost(int s0, int s1, float R, float fl, float j0, float dj) {
  if (s0 != s1) return prow_cost(s1, R, fl, j0 + dj) - prow_cost(s0, R, fl, j0);
  return s0 == PST_QUAD ? 0.5f * dj * (2.0f * j0 + dj) / R
                        : (s0 == PST_LINNEG ? -fl * dj : (s0 == PST_LINPOS ? fl * dj : 0.0f));
}

// dense in-place Cholesky of an nv x nv LDS matrix (lower triangle read and written), lanes over
// rows; and the solve with its factor (lane j holds b_j / returns x_j).  Blocked mode's Hessian.
template <int G>
__device__ void chol_dense(lfloat* A, int nv, int lane) {
  #pragma unroll 1
  for (int k = 0; k < nv; ++k) {
    float t = 0;
    if (lane >= k && lane < nv) {
      // four partial sums: the FMA chain is a quarter as long (the loads were already independent)
      float s0 = 0, s1 = 0, s2 = 0, s3 = 0;
      const lfloat *ai = A + lane * nv, *ak = A + k * nv;
      int p = 0;
      #pragma unroll 2
      for (; p + 4 <= k; p += 4) {
        s0 += ai[p] * ak[p]; s1 += ai[p + 1] * ak[p + 1];
        s2 += ai[p + 2] * ak[p + 2]; s3 += ai[p + 3] * ak[p + 3];
      }
      for (; p < k; ++p) s0 += ai[p] * ak[p];
      t = A[lane * nv + k] - ((s0 + s1) + (s2 + s3));
    }
    const float dk = gbcast<G>(t, k);
    const float lkk = sqrtf(dk > kMinVal ? dk : kMinVal);
    if (lane == k) A[k * nv + k] = lkk;
    else if (lane > k && lane < nv) A[lane * nv + k] = t / lkk;
    wsync();
  }
}
template <int G>
__device__ float chol_solve_dense(const lfloat* Lf, float x, int nv, int lane) {
  x = lane < nv ? x : 0.0f;
  #pragma unroll 1
  for (int i = 0; i < nv; ++i) {
    const float xi = gbcast<G>(x, i) / Lf[i * nv + i];
    if (lane == i) x = xi;
    else if (lane > i && lane < nv) x -= Lf[lane * nv + i] * xi;
  }
  #pragma unroll 1
  for (int i = nv - 1; i >= 0; --i) {
    const float xi = gbcast<G>(x, i) / Lf[i * nv + i];
    if (lane == i) x = xi;
    else if (lane < i) x -= Lf[i * nv + lane] * xi;
  }
  return x;
}

// Newton's Hessian in blocked mode (G = 64, one env per wave): H = M + J' diag(D) J, D_r = 1 / R_r for
// rows in the quadratic state, as the dense nv x nv lower triangle in LDS (all chol_dense reads).
// J' D J is a genuine contraction over the rows (nv up to 64 dofs, hundreds of rows in contact-rich
// scenes): one v_mfma_f32_16x16x4f32 per (16 x 16 dof tile, 4 rows), the lower-triangle tiles of
// every 4-row slice issued back to back.  Lane l feeds A[i][k] = D_r J_ri and B[k][j] = J_rj with
// i, j = tile offset + l % 16 and r = r0 + l / 16, and holds D[4 (l / 16) + v][l % 16] of the tile in
// result register v (scripts/probes/mfma16x16x4.hip checks this layout on the device).  Slices whose
// four rows are all outside the quadratic state are skipped.
__device__ __forceinline__ void hessian_mfma64(const DevModel& m, const lfloat* s, const gfloat* J, const gfloat* st,
                                               const gfloat* Rr, int nefc, lfloat* H, int lane) {
  const int nv = m.nv;
  const int col = lane & 15, kq = lane >> 4;
  v4f acc[10];
  unroll<10>([&](auto tc) { acc[decltype(tc)::value] = v4f{0.0f, 0.0f, 0.0f, 0.0f}; });
  // slices unrolled by 4 with every load of a slice independent of the others (the row's state, R
  // and its J entries), so ~24 loads per lane are in flight instead of one dependent round trip each
  #pragma unroll 4
  for (int r0 = 0; r0 < nefc; r0 += 4) {
    const int r = r0 + kq;
    const bool in = r < nefc;
    const int sr = in ? __float_as_int(st[r]) : PST_SAT;
    const float Rv = in ? (float)Rr[r] : 1.0f;
    float v[4];
    unroll<4>([&](auto bc) {
      constexpr int b = decltype(bc)::value;
      const int i = 16 * b + col;
      v[b] = (in && i < nv) ? J[r * nv + i] : 0.0f;
    });
    const float D = sr == PST_QUAD ? 1.0f / Rv : 0.0f;
    unroll<4>([&](auto ic) {
      constexpr int I = decltype(ic)::value;
      if (16 * I < nv) {
        const float a = v[I] * D;
        unroll<I + 1>([&](auto jc) {
          constexpr int Jb = decltype(jc)::value;
          constexpr int tt = I * (I + 1) / 2 + Jb;
          acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, v[Jb], acc[tt], 0, 0, 0);
        });
      }
    });
  }
  unroll<4>([&](auto ic) {
    constexpr int I = decltype(ic)::value;
    if (16 * I < nv)
      unroll<I + 1>([&](auto jc) {
        constexpr int Jb = decltype(jc)::value;
        constexpr int tt = I * (I + 1) / 2 + Jb;
        const int j = 16 * Jb + col;
        unroll<4>([&](auto vc) {
          constexpr int vv = decltype(vc)::value;
          const int i = 16 * I + 4 * kq + vv;
          if (i < nv && j < nv && i >= j) {
            float h = acc[tt][vv];
            if (m.dof_tree[i] == m.dof_tree[j]) h += s[m.L.M + midx<64>(m, i, j)];
            H[i * nv + j] = h;
          }
        });
      });
  });
}

template <int G>
__device__ float solve_primal(ENV_PARAMS, int nefc, bool newton) {
  ENV_UNPACK;
  const int nv = m.nv;
  const bool dof = lane < nv;
  const gfloat* J = scr + S.efc_J;
  const gfloat* type = scr + S.efc_type;
  const gfloat* floss = scr + S.efc_floss;
  const gfloat* Rr = scr + S.efc_R;
  const gfloat* aref = scr + S.efc_aref;
  gfloat* jar = scr + S.efc_b;
  gfloat* jv = scr + S.efc_ARii;
  gfloat* st = scr + S.efc_MJ;
  gfloat* ff = scr + S.efc_f;
  lfloat* xb = s + L.qacc;
  const float scale = m.pgs_scale;
  const float qs = dof ? s[L.qacc_smooth + lane] : 0.0f;
  const float fs = dof ? s[L.qfrc_smooth + lane] : 0.0f;
  auto is_fric = [&](int r) { return fric_like(__float_as_int(type[r]) >> 16); };
  auto is_con = [&](int r) { return (__float_as_int(type[r]) >> 16) == EFC_CONTACT; };
  const bool ell = m.cone == MRS_CONE_ELLIPTIC;  // 3-row contact blocks (floss slot: k + 1)
  // an elliptic block's zone cost at jar0 + a dj (dj null: at jar0) and its 1-D slope / curvature
  auto ell_line = [&](int r, float a, const float* dj, float& cost, float& d1, float& d2) {
    float ja[3], D[3], v[3] = {0, 0, 0};
    for (int k = 0; k < 3; ++k) {
      if (dj) v[k] = dj[k];
      ja[k] = jar[r + k] + a * v[k];
      D[k] = 1.0f / Rr[r + k];
    }
    const float ft = ell_friction(m, scr, type, r), mu = ft * rsqrtf(m.impratio);
    const int z = ell_zone(ft, m.impratio, D, ja, nullptr, &cost, nullptr);
    d1 = d2 = 0;
    if (z == PST_QUAD) {
      for (int k = 0; k < 3; ++k) { d1 += v[k] * D[k] * ja[k]; d2 += D[k] * v[k] * v[k]; }
    } else if (z == PST_CONE) {
      const float N = mu * ja[0], dN = mu * v[0];
      const float U1 = ft * ja[1], U2 = ft * ja[2], dU1 = ft * v[1], dU2 = ft * v[2];
      const float T = sqrtf(U1 * U1 + U2 * U2), dT = (U1 * dU1 + U2 * dU2) / T;
      const float Dm = D[0] / (mu * mu * (1 + mu * mu)), NT = N - mu * T, g = dN - mu * dT;
      d1 = Dm * NT * g;
      d2 = Dm * (g * g - NT * mu * ((dU1 * dU1 + dU2 * dU2) - dT * dT) / T);
    }
    return z;
  };
  // a block's cost change from jar0 to jar0 + a dj within one zone, in factored form (the plain
  // difference of two nearly equal fp32 costs can come out positive on a descent step, which the
  // solver's improvement test would take for convergence)
  auto ell_dcost = [&](int r, int z, float a, const float* dj) {
    float D[3], d[3];
    for (int k = 0; k < 3; ++k) { D[k] = 1.0f / Rr[r + k]; d[k] = a * dj[k]; }
    if (z == PST_QUAD) {
      float c = 0;
      for (int k = 0; k < 3; ++k) c += 0.5f * D[k] * d[k] * (2.0f * jar[r + k] + d[k]);
      return c;
    }
    if (z != PST_CONE) return 0.0f;
    const float ft = ell_friction(m, scr, type, r), mu = ft * rsqrtf(m.impratio);
    const float U1 = ft * jar[r + 1], U2 = ft * jar[r + 2], dU1 = ft * d[1], dU2 = ft * d[2];
    const float T0 = sqrtf(U1 * U1 + U2 * U2), T1 = sqrtf((U1 + dU1) * (U1 + dU1) + (U2 + dU2) * (U2 + dU2));
    const float dT = T0 + T1 > 0 ? (dU1 * (2.0f * U1 + dU1) + dU2 * (2.0f * U2 + dU2)) / (T0 + T1) : 0.0f;
    const float NT0 = mu * jar[r] - mu * T0, dNT = mu * d[0] - mu * dT;
    const float Dm = D[0] / (mu * mu * (1 + mu * mu));
    return 0.5f * Dm * dNT * (2.0f * NT0 + dNT);
  };
  // M[lane][k]: dense, or per kinematic tree in blocked mode (zero across trees)
  const int mytree = G == 64 && dof ? m.dof_tree[lane] : 0;
  auto mval = [&](int k) {
    if constexpr (G == 64) return m.dof_tree[k] == mytree ? (float)s[L.M + midx<G>(m, lane, k)] : 0.0f;
    else return (float)s[L.M + lane * nv + k];
  };
  lfloat* H = G == 64 ? s + L.H : s + L.L;
  // (M x)_lane
  auto mmul = [&](float x) {
    if (dof) xb[lane] = x;
    wsync();
    float y = 0;
    if (dof)
      #pragma unroll 1
      for (int k = 0; k < nv; ++k) y += mval(k) * xb[k];
    wsync();
    return y;
  };
  // out[r] = J_r x - shift * aref_r
  auto jmul = [&](float x, gfloat* out, float shift) {
    if (dof) xb[lane] = x;
    wsync();
    #pragma unroll 1
    for (int r = lane; r < nefc; r += G) {
      float v = -shift * aref[r];
      const gfloat* Jr = J + r * nv;
      // unrolled, four partial sums: the row's loads are issued together and the FMA chain is short
      float v1 = 0, v2 = 0, v3 = 0;
      int j = 0;
      #pragma unroll 2
      for (; j + 4 <= nv; j += 4) {
        v += Jr[j] * xb[j]; v1 += Jr[j + 1] * xb[j + 1];
        v2 += Jr[j + 2] * xb[j + 2]; v3 += Jr[j + 3] * xb[j + 3];
      }
      for (; j < nv; ++j) v += Jr[j] * xb[j];
      out[r] = (v + v1) + (v2 + v3);
    }
    wsync();
  };
  // mj_constraintUpdate at the stored jar: row states and forces; returns (J' f)_lane
  // (chg: some row's state differs from the one stored before)
  bool chg = false;
  auto update = [&]() {
    chg = false;
    #pragma unroll 1
    for (int r = lane; r < nefc; r += G) {
      if (ell && is_con(r) && floss[r] > 0.5f) {
        // elliptic block: the first row's lane sets the zone and the forces of all three rows (the
        // middle zone's Hessian depends on jar, so a block in it always counts as changed)
        if (floss[r] != 1.0f) continue;
        float ja3[3], D[3], f3[3];
        for (int k = 0; k < 3; ++k) { ja3[k] = jar[r + k]; D[k] = 1.0f / Rr[r + k]; }
        const int z = ell_zone(ell_friction(m, scr, type, r), m.impratio, D, ja3, f3, nullptr, nullptr);
        chg |= __float_as_int(st[r]) != z || z == PST_CONE;
        for (int k = 0; k < 3; ++k) { st[r + k] = __int_as_float(z); ff[r + k] = f3[k]; }
        continue;
      }
      const float R = Rr[r], fl = floss[r], ja = jar[r];
      const int stt = prow_state(is_fric(r), R, fl, ja);
      chg |= __float_as_int(st[r]) != stt;
      st[r] = __int_as_float(stt);
      ff[r] = -prow_slope(stt, R, fl, ja);
    }
    wsync();
    float q = 0;
    if (dof) {
      float q1 = 0, q2 = 0, q3 = 0;
      int r = 0;
      #pragma unroll 2
      for (; r + 4 <= nefc; r += 4) {
        q += J[r * nv + lane] * ff[r]; q1 += J[(r + 1) * nv + lane] * ff[r + 1];
        q2 += J[(r + 2) * nv + lane] * ff[r + 2]; q3 += J[(r + 3) * nv + lane] * ff[r + 3];
      }
      for (; r < nefc; ++r) q += J[r * nv + lane] * ff[r];
      q = (q + q1) + (q2 + q3);
    }
    return q;
  };
  // total cost at x (warm-start selection); leaves J x - aref in jar.  The Gauss term is
  // 1/2 (x - qs)' M (x - qs), formed from the difference (fp32: no cancellation of M x - M qs)
  auto cost_at = [&](float x) {
    const float md = mmul(x - qs);
    jmul(x, jar, 1.0f);
    float c = 0;
    #pragma unroll 1
    for (int r = lane; r < nefc; r += G) {
      if (ell && is_con(r) && floss[r] > 0.5f) {
        if (floss[r] == 1.0f) {
          float cb, d1, d2;
          ell_line(r, 0.0f, nullptr, cb, d1, d2);
          c += cb;
        }
        continue;
      }
      const float R = Rr[r], fl = floss[r], ja = jar[r];
      c += prow_cost(prow_state(is_fric(r), R, fl, ja), R, fl, ja);
    }
    return gsum<G>((dof ? 0.5f * md * (x - qs) : 0.0f) + c);
  };

  float qa = qs;
  if (!(m.disableflags & MRS_DSBL_WARMSTART)) {
    const float xw = dof ? s[L.qacc_ws + lane] : 0.0f;
    const float c_ws = cost_at(xw), c_sm = cost_at(qs);
    if (c_ws <= c_sm) qa = xw;
  }
  // Md = M (qacc - qacc_smooth) = M qacc - qfrc_smooth, carried as a difference
  float Md = mmul(qa - qs);
  jmul(qa, jar, 1.0f);
  float qfrc = update();
  float p = 0, gold = 0, Mgold = 0;
  bool refined = false;
  // the Hessian's factor in H is still that of the current row states (refinement step after a step
  // that kept the active set): H = M + J'DJ depends on the states only, so it is not rebuilt
  bool reuse = false;
  int nit = 0;  // steps taken (mjData.solver_niter)
  #pragma unroll 1
  for (int iter = 0;; ++iter) {
    const float grad = dof ? Md - qfrc : 0.0f;
    float Mg;
    if (newton && reuse) {
      if constexpr (G == 64) {
        Mg = chol_solve_dense<G>(H, grad, nv, lane);
      } else {
        MRS_CALL(G, Mg = chol_solve_lanes<G>(mp, H, grad, lane));
      }
    } else if (newton) {
      // H row `lane` (dense: into the factor slot L.L; blocked: L.H, by MFMA), then factor in place
      unsigned long long t_h = SUB_T();
      if constexpr (G == 64) {
        hessian_mfma64(m, s, J, st, Rr, nefc, H, lane);
      } else {
        if (dof)
          #pragma unroll 1
          for (int k = 0; k < nv; ++k) {
            float h = mval(k);
            #pragma unroll 1
            for (int r = 0; r < nefc; ++r)
              if (__float_as_int(st[r]) == PST_QUAD) h += J[r * nv + lane] * J[r * nv + k] / Rr[r];
            H[lane * nv + k] = h;
          }
      }
      wsync();
      if (ell) {
        // elliptic blocks in the middle zone: J_b' H_b J_b with the zone's 3x3 jar-space Hessian
        // (bottom-zone blocks are quadratic rows, already in); lower triangle, lane per H row
        #pragma unroll 1
        for (int r = 0; r < nefc; ++r) {
          if (!(is_con(r) && floss[r] == 1.0f) || __float_as_int(st[r]) != PST_CONE) continue;
          float ja3[3], D[3], Hb[9];
          for (int k = 0; k < 3; ++k) { ja3[k] = jar[r + k]; D[k] = 1.0f / Rr[r + k]; }
          ell_zone(ell_friction(m, scr, type, r), m.impratio, D, ja3, nullptr, nullptr, Hb);
          if (dof) {
            float u[3];  // (H_b J_b)[:, lane]
            for (int a = 0; a < 3; ++a)
              u[a] = Hb[3 * a] * J[r * nv + lane] + Hb[3 * a + 1] * J[(r + 1) * nv + lane] + Hb[3 * a + 2] * J[(r + 2) * nv + lane];
            #pragma unroll 1
            for (int k = 0; k <= (G == 64 ? lane : nv - 1); ++k)
              H[lane * nv + k] += u[0] * J[r * nv + k] + u[1] * J[(r + 1) * nv + k] + u[2] * J[(r + 2) * nv + k];
          }
          wsync();
        }
      }
      SUB_ADD(PH_CON_DEL, t_h);
      t_h = SUB_T();
      if constexpr (G == 64) {
        chol_dense<G>(H, nv, lane);
        Mg = chol_solve_dense<G>(H, grad, nv, lane);
        SUB_ADD(PH_CON_WARM, t_h);
      } else {
        MRS_CALL(G, cholesky<G>(mp, H, H, lane));
        MRS_CALL(G, Mg = chol_solve_lanes<G>(mp, H, grad, lane));
      }
    } else {
      MRS_CALL(G, Mg = chol_solve_lanes<G>(mp, s + L.L, grad, lane));
    }
    if (iter == 0 || newton) {
      p = -Mg;
    } else {
      // Polak-Ribiere, reset when negative
      const float num = gsum<G>(grad * (Mg - Mgold)), den = gsum<G>(gold * Mgold);
      const float beta = fmaxf(0.0f, num / (den > kMinVal ? den : kMinVal));
      p = -Mg + beta * p;
    }
    if (iter >= m.iterations) break;
    const float Mv = mmul(p);
    jmul(p, jv, 0.0f);
    // exact line search: safeguarded Newton on the 1-D piecewise quadratic
    const float g1 = gsum<G>(p * Md), g2 = gsum<G>(p * Mv), snorm = sqrtf(gsum<G>(p * p));
    auto ls_eval = [&](float a, float a0, float& d1, float& d2, bool& ch) {
      float s1 = 0, s2 = 0;
      bool c = false;
      #pragma unroll 1
      for (int r = lane; r < nefc; r += G) {
        if (ell && is_con(r) && floss[r] > 0.5f) {
          // elliptic block: the middle zone is not quadratic in a, so a step ending in it is never
          // taken as exact
          if (floss[r] == 1.0f) {
            const float dj[3] = {jv[r], jv[r + 1], jv[r + 2]};
            float cb, e1, e2, x1, x2;
            const int z = ell_line(r, a, dj, cb, e1, e2);
            const int z0 = ell_line(r, a0, dj, cb, x1, x2);
            c |= z != z0 || z == PST_CONE;
            s1 += e1;
            s2 += e2;
          }
          continue;
        }
        const float v = jv[r];
        if (v == 0) continue;
        const bool fr = is_fric(r);
        const float R = Rr[r], fl = floss[r], j0 = jar[r], ja = j0 + a * v;
        const int stt = prow_state(fr, R, fl, ja);
        c |= stt != prow_state(fr, R, fl, j0 + a0 * v);
        s1 += v * prow_slope(stt, R, fl, ja);
        if (stt == PST_QUAD) s2 += v * v / R;
      }
      d1 = g1 + a * g2 + gsum<G>(s1);
      d2 = g2 + gsum<G>(s2);
      ch = gany<G>(c);
    };
    float alpha = 0;
    if (snorm >= kMinVal && g2 > 0) {
      const float gtol = m.tolerance * m.ls_tolerance * snorm / scale;
      float d1, d2;
      bool ch;
      ls_eval(0.0f, 0.0f, d1, d2, ch);
      if (d1 < 0) {
        float a = 0, lo = 0, hi = -1;
        #pragma unroll 1
        for (int it = 0; it < m.ls_iterations; ++it) {
          float an = a - d1 / d2;
          bool nstep = true;
          if (hi >= 0 && (an <= lo || an >= hi)) { an = 0.5f * (lo + hi); nstep = false; }
          float n1, n2;
          ls_eval(an, a, n1, n2, ch);
          a = an; d1 = n1; d2 = n2;
          if (fabsf(d1) < gtol || (nstep && !ch)) break;
          if (d1 < 0) lo = a; else hi = a;
        }
        alpha = a;
      }
    }
    if (alpha == 0) break;
    // cost decrease of the step from per-row differences; rows move to the new point
    float dc = 0;
    bool changed = false;
    #pragma unroll 1
    for (int r = lane; r < nefc; r += G) {
      if (ell && is_con(r) && floss[r] > 0.5f) {
        if (floss[r] == 1.0f) {
          const float dj[3] = {jv[r], jv[r + 1], jv[r + 2]};
          float c0, c1, d1, d2;
          const int z0 = ell_line(r, 0.0f, nullptr, c0, d1, d2);
          const int z1 = ell_line(r, alpha, dj, c1, d1, d2);
          dc += z0 == z1 ? ell_dcost(r, z0, alpha, dj) : c1 - c0;
          changed |= z1 != __float_as_int(st[r]) || z1 == PST_CONE;
          for (int k = 0; k < 3; ++k) jar[r + k] = jar[r + k] + alpha * dj[k];
        }
        continue;
      }
      const bool fr = is_fric(r);
      const float R = Rr[r], fl = floss[r], j0 = jar[r], j1 = j0 + alpha * jv[r];
      const int s0 = __float_as_int(st[r]), s1 = prow_state(fr, R, fl, j1);
      dc += prow_dcost(s0, s1, R, fl, j0, alpha * jv[r]);
      changed |= s0 != s1;
      jar[r] = j1;
    }
    const float dcost = alpha * g1 + 0.5f * alpha * alpha * g2 + gsum<G>(dc);
    changed = gany<G>(changed);
    qa += alpha * p;
    Md += alpha * Mv;
    gold = grad;
    Mgold = Mg;
    wsync();
    qfrc = update();
    ++nit;
    const float gn = dof ? Md - qfrc : 0.0f;
    const float gnorm = sqrtf(gsum<G>(gn * gn));
    if (scale * -dcost < m.tolerance || scale * gnorm < m.tolerance) break;
    // H = M + J'DJ depends on the row states only: after a step that kept them, the next Newton step
    // reuses its factor (mj_solNewton keeps iterating until the tests above stop it)
    reuse = newton && !changed;
    if (newton && !changed && (m.restate & MRS_RESTATE_NEWTON_REFINE)) {
      // opt-in (not upstream): the step solved the quadratic model up to the fp32 factor's rounding
      // (cond(H) eps |grad|); one refinement step from fresh residuals, then stop (oracle.c) -- unless
      // the residual is already at the rounding level of the gradient's own terms
      const bool floor = fabsf(gn) <= 64.0f * __FLT_EPSILON__ * (fabsf(Md) + fabsf(qfrc));
      if (refined || !gany<G>(!floor)) break;
      refined = true;
      Md = mmul(qa - qs);
      jmul(qa, jar, 1.0f);
      qfrc = update();
      reuse = !gany<G>(chg);
    }
  }
  if (dof) s[L.qfrc_con + lane] = qfrc;
  if (lane == 0) s[L.niter] = __int_as_float(nit);
  wsync();
  return dof ? qa : 0.0f;
}

// The same primal solvers (solve_primal's algorithm, step for step) for small systems on G = 16
// groups (nv <= 16, nefc <= 16), register-resident: lane j holds column j of every row of J and dof
// j of the vectors, lane r holds row r's scalars (R, aref, friction-loss bound, jar = J_r qacc - aref,
// J_r p, state, force).  Row products J x are KR independent DPP row reductions, J' f and M x are
// DPP row broadcasts and FMAs, so nothing but the Hessian's factor (LDS, as in solve_primal) leaves
// the registers -- the generic form keeps the rows and their products in the env's global scratch,
// one dependent global round trip per row loop, and that was half of the reference scene's step
// under MuJoCo's default solver.  KR: rows unrolled (the wave's largest system rounded up), KV: dof
// unroll bound (>= nv).  Rows past the group's nefc are zero rows (J = 0, aref = 0): jar = 0 keeps
// them satisfied, so they add nothing to any cost, slope or force.
// kUnit: every row is the unit vector of the dof in lane r's `mydof` (dof friction-loss rows), built
// in registers instead of read from the global rows J (row forces then stored only for force sensors)
template <bool kUnit, int KR, int KV>
__device__ __forceinline__ float primal_small16(ENV_PARAMS, const gfloat* J, gfloat* ff, int nefc, float myR, float myaref,
                                                float myfl, bool myfric, float qs, bool newton, int mydof = -1) {
  constexpr int G = 16;
  ENV_UNPACK;
  const int nv = m.nv;
  const bool dof = lane < nv;
  const bool row = kUnit ? myfric : lane < nefc;
  if (!row) { myR = 1; myaref = 0; myfl = 0; myfric = false; }
  qs = dof ? qs : 0.0f;
  float Jt[KR];
  unroll<KR>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    if constexpr (kUnit)
      Jt[r] = 0.0f;  // (unused: the unit rows' products are lane-local)
    else
      Jt[r] = (r < nefc && dof) ? J[r * nv + lane] : 0.0f;
  });
  // row `lane` of M (LDS; zero past nv, where x is zero too)
  auto mrow = [&](int k) { return (k < nv && dof) ? (float)s[L.M + lane * nv + k] : 0.0f; };
  const float scale = m.pgs_scale;
  // lane r: J_r x (KR independent row reductions)
  auto rows_dot = [&](float x) {
    float out = 0;
    if constexpr (kUnit) {
      out = row ? x : 0.0f;
    } else {
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        const float t = gsum<16>(Jt[r] * x);
        if (lane == r) out = t;
      });
    }
    return out;
  };
  // lane j: (M x)_j, (J' f)_j
  auto mmul = [&](float x) {
    float y = 0;
    unroll<KV>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      y += mrow(k) * rowb<k>(x);
    });
    return y;
  };
  auto jtmul = [&](float f) {
    float q = 0;
    if constexpr (kUnit) {
      q = row ? f : 0.0f;
    } else {
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        q += Jt[r] * rowb<r>(f);
      });
    }
    return q;
  };
  float jar = 0, myf = 0;  // row lanes
  int st = PST_SAT;
  // mj_constraintUpdate at jar: row state and force, returns (J' f)_lane
  auto update = [&]() {
    st = row ? prow_state(myfric, myR, myfl, jar) : PST_SAT;
    myf = row ? -prow_slope(st, myR, myfl, jar) : 0.0f;
    return jtmul(myf);
  };
  auto cost_at = [&](float x) {
    const float md = mmul(x - qs);
    jar = rows_dot(x) - myaref;
    const float c = row ? prow_cost(prow_state(myfric, myR, myfl, jar), myR, myfl, jar) : 0.0f;
    return gsum<16>((dof ? 0.5f * md * (x - qs) : 0.0f) + c);
  };
  float qa = qs;
  if (!(m.disableflags & MRS_DSBL_WARMSTART)) {
    const float xw = dof ? s[L.qacc_ws + lane] : 0.0f;
    const float c_ws = cost_at(xw), c_sm = cost_at(qs);
    if (c_ws <= c_sm) qa = xw;
  }
  float Md = mmul(qa - qs);
  jar = rows_dot(qa) - myaref;
  float qfrc = update();
  float p = 0, gold = 0, Mgold = 0;
  bool refined = false, reuse = false;  // reuse: H's factor is that of the current row states
  int nit = 0;
  lfloat* H = s + L.L;
  #pragma unroll 1
  for (int iter = 0;; ++iter) {
    const float grad = dof ? Md - qfrc : 0.0f;
    float Mg;
    if (newton && reuse) {
      MRS_CALL(16, Mg = chol_solve_lanes<16>(mp, H, grad, lane));
    } else if (newton) {
      // H = M + J' diag(D of quadratic rows) J, row `lane` in registers, then factored in the LDS
      // factor slot (M's factor is not needed again before integrate() refactors)
      const float Dr = (row && st == PST_QUAD) ? 1.0f / myR : 0.0f;
      float dj[KR];
      unroll<KR>([&](auto rc) {
        constexpr int r = decltype(rc)::value;
        dj[r] = kUnit ? 0.0f : Jt[r] * rowb<r>(Dr);
      });
      unroll<KV>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        float h = mrow(k);
        if constexpr (kUnit) {
          if (lane == k) h += Dr;  // J' D J of unit rows: diagonal
        } else {
          unroll<KR>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            h += dj[r] * rowb<k>(Jt[r]);
          });
        }
        if (dof && k < nv) H[lane * nv + k] = h;
      });
      wsync();
      MRS_CALL(16, cholesky<16>(mp, H, H, lane));
      MRS_CALL(16, Mg = chol_solve_lanes<16>(mp, H, grad, lane));
    } else {
      MRS_CALL(16, Mg = chol_solve_lanes<16>(mp, s + L.L, grad, lane));
    }
    if (iter == 0 || newton) {
      p = -Mg;
    } else {
      const float num = gsum<16>(grad * (Mg - Mgold)), den = gsum<16>(gold * Mgold);
      const float beta = fmaxf(0.0f, num / (den > kMinVal ? den : kMinVal));
      p = -Mg + beta * p;
    }
    if (iter >= m.iterations) break;
    const float Mv = mmul(p);
    const float jv = rows_dot(p);
    const float g1 = gsum<16>(p * Md), g2 = gsum<16>(p * Mv), snorm = sqrtf(gsum<16>(p * p));
    auto ls_eval = [&](float a, float a0, float& d1, float& d2, bool& ch) {
      float s1 = 0, s2 = 0;
      bool c = false;
      if (row && jv != 0) {
        const float ja = jar + a * jv;
        const int stt = prow_state(myfric, myR, myfl, ja);
        c = stt != prow_state(myfric, myR, myfl, jar + a0 * jv);
        s1 = jv * prow_slope(stt, myR, myfl, ja);
        if (stt == PST_QUAD) s2 = jv * jv / myR;
      }
      d1 = g1 + a * g2 + gsum<16>(s1);
      d2 = g2 + gsum<16>(s2);
      ch = gany<16>(c);
    };
    float alpha = 0;
    if (snorm >= kMinVal && g2 > 0) {
      const float gtol = m.tolerance * m.ls_tolerance * snorm / scale;
      float d1, d2;
      bool ch;
      ls_eval(0.0f, 0.0f, d1, d2, ch);
      if (d1 < 0) {
        float a = 0, lo = 0, hi = -1;
        #pragma unroll 1
        for (int it = 0; it < m.ls_iterations; ++it) {
          float an = a - d1 / d2;
          bool nstep = true;
          if (hi >= 0 && (an <= lo || an >= hi)) { an = 0.5f * (lo + hi); nstep = false; }
          float n1, n2;
          ls_eval(an, a, n1, n2, ch);
          a = an; d1 = n1; d2 = n2;
          if (fabsf(d1) < gtol || (nstep && !ch)) break;
          if (d1 < 0) lo = a; else hi = a;
        }
        alpha = a;
      }
    }
    if (alpha == 0) break;
    float dc = 0;
    bool changed = false;
    if (row) {
      const float j1 = jar + alpha * jv;
      const int s1 = prow_state(myfric, myR, myfl, j1);
      dc = prow_dcost(st, s1, myR, myfl, jar, alpha * jv);
      changed = st != s1;
      jar = j1;
    }
    const float dcost = alpha * g1 + 0.5f * alpha * alpha * g2 + gsum<16>(dc);
    changed = gany<16>(changed);
    qa += alpha * p;
    Md += alpha * Mv;
    gold = grad;
    Mgold = Mg;
    qfrc = update();
    ++nit;
    const float gn = dof ? Md - qfrc : 0.0f;
    const float gnorm = sqrtf(gsum<16>(gn * gn));
    if (scale * -dcost < m.tolerance || scale * gnorm < m.tolerance) break;
    reuse = newton && !changed;  // (solve_primal)
    if (newton && !changed && (m.restate & MRS_RESTATE_NEWTON_REFINE)) {
      const bool floor = fabsf(gn) <= 64.0f * __FLT_EPSILON__ * (fabsf(Md) + fabsf(qfrc));
      if (refined || !gany<16>(!floor)) break;
      refined = true;
      Md = mmul(qa - qs);
      jar = rows_dot(qa) - myaref;
      const int st_old = st;
      qfrc = update();
      reuse = !gany<16>(st != st_old);
    }
  }
  if (dof) s[L.qfrc_con + lane] = qfrc;
  if (row && (!kUnit || (m.acc_sens & 2))) ff[kUnit ? mydof : lane] = myf;  // row forces (mj_rnePostConstraint, mrs_batch_get_efc)
  if (lane == 0) s[L.niter] = __int_as_float(nit);
  wsync();
  return dof ? qa : 0.0f;
}

template <int G, bool kPrimal = false, bool kHot = false>
__device__ float constraints_dense(ENV_PARAMS, int ncon, float qacc_s, int pre_nefc = -1);
template <int G>
__device__ int dense_rows(ENV_PARAMS, int ncon);

template <int G, bool kPrimal = false, bool kHot = false>
__device__ MRS_PHASE float constraints(ENV_PARAMS, int ncon, float qacc_s, int pre_nefc = -1) {
  ENV_UNPACK;
  if constexpr (G == 64) {
    if (m.solver != MRS_SOL_PGS || m.cone == MRS_CONE_ELLIPTIC || m.xrows > 0) {
      // Newton / CG in blocked mode, elliptic cones, equality and tendon rows under every solver:
      // dense rows (solve_primal, or the row-serial PGS with its 3-row contact blocks)
      float qa;
      [[clang::noinline]] qa = constraints_dense<G>(ENV_ARGS, ncon, qacc_s);
      return qa;
    }
    switch (m.pipe_w) {
      case 8: return constraints_sparse<8>(ENV_ARGS, ncon, qacc_s);
      case 16: {
        // out of line the call saves and restores ~106 callee-saved VGPRs through scratch memory
        // every step (C5: ~2 GB per 10-step launch); inlined, the kernel's own live values spill
        // around the solve instead and the launch was measured slower (12.0 vs 10.6 ms), so it stays
        // out of line unless MRS_SPARSE_INLINE (A/B builds)
        float qa;
#ifdef MRS_SPARSE_INLINE
        [[clang::always_inline]] qa = constraints_sparse<16>(ENV_ARGS, ncon, qacc_s);
#else
        qa = constraints_sparse<16>(ENV_ARGS, ncon, qacc_s);
#endif
        return qa;
      }
      case 32: return constraints_sparse<32>(ENV_ARGS, ncon, qacc_s);
      default: return constraints_sparse<64>(ENV_ARGS, ncon, qacc_s);
    }
  }
  const int nv = m.nv;
  if (m.disableflags & MRS_DSBL_CONSTRAINT) { if (lane < nv) s[L.qfrc_con + lane] = 0; wsync(); return qacc_s; }
  if constexpr (G == 16) {
    // Friction-loss rows only (no contact, no active joint limit: C3's steady state): every row is
    // the unit vector of its dof, so lane r builds row r's scalars from the model and the LDS state
    // and the register-resident PGS builds J itself -- no row goes through the global scratch.
    const int nf = (m.disableflags & MRS_DSBL_FRICTIONLOSS) ? 0 : m.nfric;
    bool lim = false;
    if (!(m.disableflags & MRS_DSBL_LIMIT))
      #pragma unroll 1
      for (int k = lane; k < m.nlim; k += G) {
        const lfloat* lr = shared_lds(m) + m.shr_lim + 4 * k;  // qpos address, margin, range
        const float q = s[L.qpos + __float_as_int(lr[0])], mg = lr[1];
        lim |= (q - lr[2] < mg) | (lr[3] - q < mg);
      }
    // (kPrimal: the G = 16 kernel instantiated for models whose solver is Newton or CG, so the
    // primal form is inlined only there and the PGS kernels keep their code and registers)
    if ((kPrimal ? m.solver != MRS_SOL_PGS : m.solver == MRS_SOL_PGS) && ncon == 0 && nf > 0 && nf <= 16 &&
        m.xrows == 0 && !gany<G>(lim)) {
      if (lane == 0) scr[S.efc_n] = __int_as_float(-1);  // rows stay in registers
      // rows indexed by dof: lane j holds the friction-loss row of dof j, if it has one (its index in
      // the efc order from the dof table, batch.hip dofrec[13]); the rows' order is the dof order,
      // mj_makeConstraint's, and every group of the wave has the same rows (one model)
      int myk = -1;
      float myR = 1, myaref = 0, myb = 0, myfl = 0;
      if (lane < nv) {
        myk = __float_as_int(dof_tab<G>(m, lane)[13]);
        if (myk >= 0) {
          // the row's model constants from workgroup LDS (batch.hip fricrec: dof, R, B, frictionloss)
          const lfloat* fr = shared_lds(m) + m.shr_fric + 4 * myk;
          myR = fr[1];
          myaref = -fr[2] * s[L.qvel + lane];  // friction rows have no position term
          myb = s[L.qacc_smooth + lane] - myaref;
          myfl = fr[3];
        }
      }
      const unsigned fmask = static_cast<unsigned>(__ballot(myk >= 0)) & 0xffffu;
      float qa;
      if constexpr (kPrimal) {
        // Newton / CG (MuJoCo's default solver): the register-resident primal form on the same rows
        const bool newton = m.solver == MRS_SOL_NEWTON;
        // (a 4-wide form for nv <= 4 measured the same on C2: 164.7 vs 165.0 M)
        if (m.nv <= 8)
          qa = primal_small16<true, 8, 8>(ENV_ARGS, nullptr, scr + S.efc_f, nf, myR, myaref, myfl, myk >= 0, qacc_s, newton, myk);
        else
          qa = primal_small16<true, 16, 16>(ENV_ARGS, nullptr, scr + S.efc_f, nf, myR, myaref, myfl, myk >= 0, qacc_s, newton, myk);
        return qa;
      }
      // dofs unrolled to 8 when the model has at most 8: a quarter of the substitution code
      if (m.nv <= 8)
        qa = pgs_small16_qacc<true, 8>(m, s, nullptr, scr + S.efc_f, nf, 8, myR, myaref, myb, myfl, qacc_s, lane, myk, fmask);
      else
        qa = pgs_small16_qacc<true, 16>(m, s, nullptr, scr + S.efc_f, nf, 16, myR, myaref, myb, myfl, qacc_s, lane, myk, fmask);
      wsync();
      return qa;
    }
  }
  // rows with contacts or active joint limits: the dense row path, out of line -- cold in C3's
  // steady state, and keeping it out of the inlined step loop keeps the hot code footprint small
  float qa;
#ifdef MRS_DENSE_INLINE_HOT
  if constexpr (kHot) {
    [[clang::always_inline]] qa = constraints_dense<G, kPrimal, kHot>(ENV_ARGS, ncon, qacc_s, pre_nefc);
    return qa;
  }
#endif
  [[clang::noinline]] qa = constraints_dense<G, kPrimal, kHot>(ENV_ARGS, ncon, qacc_s, pre_nefc);
  return qa;
}

// dense constraint rows in the env's global scratch (J, M^-1 J', row scalars), then the
// register-resident PGS (<= 16 rows on G = 16) or the row-serial PGS with wave reductions
// mj_makeImpedance of row r (mj_makeConstraint's rows in the env's scratch): its regulariser R and
// reference acceleration aref = -B J qvel - K imp (pos - margin), from the row's type, distance and
// model parameters.  The dense solve's set-up and the helper waves (dense_impedance) share it.
template <int G>
__device__ __forceinline__ void row_impedance(const DevModel& m, const lfloat* s, const gfloat* scr, int r, float& R_out,
                                              float& aref_out) {
  const LdsLayout& L = m.L;
  const ScratchLayout& S = m.S;
  const int nv = m.nv;
  const gfloat* J = scr + S.efc_J;
  const gfloat* type = scr + S.efc_type;
  const gfloat* pos = scr + S.efc_pos;
  const gfloat* marg = scr + S.efc_margin;
  const gfloat* floss = scr + S.efc_floss;
  const gfloat* bb = scr + S.efc_b;
  const int code = __float_as_int(type[r]);
  const int t = code >> 16, id = code & 0xffff;
  CPtr<float> sr, si;
  float diag;
  if (t == EFC_FRICTION) { sr = m.dof_solref + 2 * id; si = m.dof_solimp + 5 * id; diag = m.dof_invweight0[id]; }
  else if (t == EFC_EQUALITY) { sr = m.eq_solref + 2 * id; si = m.eq_solimp + 5 * id; diag = bb[r]; }
  else if (t == EFC_LIMIT) { sr = m.jnt_solref + 2 * id; si = m.jnt_solimp + 5 * id; diag = m.dof_invweight0[m.jnt_dofadr[id]]; }
  else if (t == EFC_TFRICTION) { sr = m.ten_solref_fri + 2 * id; si = m.ten_solimp_fri + 5 * id; diag = m.ten_prm[12 * id + 8]; }
  else if (t == EFC_TLIMIT) { sr = m.ten_solref_lim + 2 * id; si = m.ten_solimp_lim + 5 * id; diag = m.ten_prm[12 * id + 8]; }
  else {
    const gfloat* rec = scr + S.con + kConRec * id;
    const int p = __float_as_int(rec[0]);
    sr = m.pair_solref + 2 * p; si = m.pair_solimp + 5 * p;
    const int b1 = m.geom_bodyid[m.pair_g1[p]], b2 = m.geom_bodyid[m.pair_g2[p]];
    float tran = m.body_invweight0[2 * b1] + m.body_invweight0[2 * b2];
    diag = tran;
    if (m.pair_dim[p] == 3 && m.cone == MRS_CONE_ELLIPTIC) {
      // elliptic: diagApprox tran for every row of the block, the tangents' regulariser / impratio
      if (floss[r] > 1.5f) diag = tran / m.impratio;
    } else if (m.pair_dim[p] == 3) {
      // pyramid edge: diagApprox tran (1 + mu^2) (mu sliding, for both tangent directions);
      // mj_makeImpedance scales the edges' regulariser by 2 mu^2 / impratio
      const float mu = m.pair_friction[3 * p];
      diag = tran * (1 + mu * mu) * (2 * mu * mu / m.impratio);
    }
  }
  const float imp = impedance(si, pos[r], marg[r]);
  float R = (1 - imp) * diag / imp;
  R = R > kMinVal ? R : kMinVal;
  const float dmax = clampf(si[1], 0.0001f, 0.9999f);
  float K, B;
  if (sr[0] > 0) {
    float tc = sr[0], dr = sr[1];
    if (!(m.disableflags & MRS_DSBL_REFSAFE) && tc < 2 * m.timestep) tc = 2 * m.timestep;
    K = 1 / (dmax * dmax * tc * tc * dr * dr);
    B = 2 / (dmax * tc);
  } else {
    K = -sr[0] / (dmax * dmax);
    B = -sr[1] / dmax;
  }
  float vel = 0;
  const gfloat* Jr = J + r * nv;
  #pragma unroll 4
  for (int j = 0; j < nv; ++j) vel += Jr[j] * s[L.qvel + j];
  // (friction-loss rows and the tangent rows of an elliptic block carry no position term)
  const float pterm = (t == EFC_FRICTION || t == EFC_TFRICTION || (t == EFC_CONTACT && floss[r] > 1.5f))
                          ? 0.0f : K * imp * (pos[r] - marg[r]);
  R_out = R;
  aref_out = -B * vel - pterm;
}

// the helper waves' share of the dense set-up (step_kernel): R and aref of every row into the scratch
template <int G>
__device__ __forceinline__ void dense_impedance(ENV_PARAMS, int nefc) {
  ENV_UNPACK;
  #pragma unroll 1
  for (int r = lane; r < nefc; r += G) {
    float R, ar;
    row_impedance<G>(m, s, scr, r, R, ar);
    scr[S.efc_R + r] = R;
    scr[S.efc_aref + r] = ar;
  }
  wsync();
}

// mj_makeConstraint's rows into the env's scratch (dense J, type, pos, margin, friction-loss bound;
// contact records' first-row index): equality, friction loss, limits, contacts; returns nefc (also
// in scr[S.efc_n]).  Reads kinematics, com_pos (cdof, subtree coms) and, for tendon limits, the
// step's tendon lengths (smooth_forces)
template <int G>
__device__ int dense_rows(ENV_PARAMS, int ncon) {
  ENV_UNPACK;
  if constexpr (G == 64) ncon = uniform_int(ncon);
  const int nv = m.nv;
  gfloat* J = scr + S.efc_J;
  gfloat* type = scr + S.efc_type;
  gfloat* pos = scr + S.efc_pos;
  gfloat* marg = scr + S.efc_margin;
  gfloat* floss = scr + S.efc_floss;
  gfloat* bb = scr + S.efc_b;
  int nefc = 0;
  // solref/solimp/diagApprox per row are re-derived from (type, id) when computing impedance;
  // keep ids in a small per-row int array inside the type slot (type*65536 + id)
  // --- equality rows, first as mj_makeConstraint orders them (oracle.c equality_rows: connect and
  // weld anchor points, weld's rotation error imag(conj(q1 relquat) q2) * torquescale with its exact
  // derivative per dof, joint polynomial couplings); each row's diagApprox goes to the b slot until
  // the impedance pass reads it
  #pragma unroll 1
  for (int q = 0; q < m.neq; ++q) {
    const int t = m.eq_type[q], o1 = m.eq_obj1id[q], o2 = m.eq_obj2id[q];
    const CPtr<float> dd = m.eq_data + MRS_NEQDATA * q;
    const int code = EFC_EQUALITY * 65536 + q;
    if (t == MRS_EQ_JOINT) {
      const int d1 = m.jnt_dofadr[o1];
      const float x1 = s[L.qpos + m.jnt_qposadr[o1]] - dd[5];
      float poly = dd[0], dpoly = 0, diag = m.dof_invweight0[d1];
      int d2 = -1;
      if (o2 >= 0) {
        d2 = m.jnt_dofadr[o2];
        const float x = s[L.qpos + m.jnt_qposadr[o2]] - dd[6];
        poly = dd[0] + x * (dd[1] + x * (dd[2] + x * (dd[3] + x * dd[4])));
        dpoly = dd[1] + x * (2 * dd[2] + x * (3 * dd[3] + x * 4 * dd[4]));
        diag += m.dof_invweight0[d2];
      }
      if (lane < nv) J[nefc * nv + lane] = (lane == d1 ? 1.0f : 0.0f) - (lane == d2 ? dpoly : 0.0f);
      if (lane == 0) {
        type[nefc] = __int_as_float(code);
        pos[nefc] = x1 - poly; marg[nefc] = 0; floss[nefc] = kEqBound; bb[nefc] = diag;
      }
      ++nefc;
      continue;
    }
    float x1[3] = {0, 0, 0}, x2[3] = {0, 0, 0}, q1[4] = {1, 0, 0, 0}, q2[4] = {1, 0, 0, 0};
    if (o1 > 0) {
      for (int i = 0; i < 3; ++i) x1[i] = s[L.xpos + 3 * o1 + i];
      for (int i = 0; i < 4; ++i) q1[i] = s[L.xquat + 4 * o1 + i];
    }
    if (o2 > 0) {
      for (int i = 0; i < 3; ++i) x2[i] = s[L.xpos + 3 * o2 + i];
      for (int i = 0; i < 4; ++i) q2[i] = s[L.xquat + 4 * o2 + i];
    }
    float l1[3], l2[3];
    if (t == MRS_EQ_CONNECT) {
      for (int i = 0; i < 3; ++i) { l1[i] = dd[i]; l2[i] = dd[3 + i]; }
    } else {
      const float an[3] = {dd[0], dd[1], dd[2]}, rq[4] = {dd[6], dd[7], dd[8], dd[9]};
      float ra[3];
      rot_quat(ra, an, rq);
      for (int i = 0; i < 3; ++i) { l2[i] = an[i]; l1[i] = dd[3 + i] + ra[i]; }
    }
    float p1[3], p2[3], rr[3];
    rot_quat(rr, l1, q1);
    for (int i = 0; i < 3; ++i) p1[i] = x1[i] + rr[i];
    rot_quat(rr, l2, q2);
    for (int i = 0; i < 3; ++i) p2[i] = x2[i] + rr[i];
    float c1[3] = {0, 0, 0}, c2[3] = {0, 0, 0};
    if (lane < nv) {
      jac_col(m, s, o1, p1, lane, c1);
      jac_col(m, s, o2, p2, lane, c2);
    }
    const float tdiag = m.body_invweight0[2 * o1] + m.body_invweight0[2 * o2];
    for (int k = 0; k < 3; ++k) {
      if (lane < nv) J[nefc * nv + lane] = c1[k] - c2[k];
      if (lane == 0) {
        type[nefc] = __int_as_float(code);
        pos[nefc] = p1[k] - p2[k]; marg[nefc] = 0; floss[nefc] = kEqBound; bb[nefc] = tdiag;
      }
      ++nefc;
    }
    if (t != MRS_EQ_WELD) continue;
    const float ts = dd[10], rq[4] = {dd[6], dd[7], dd[8], dd[9]};
    float q1r[4], cq[4], e[4];
    quat_mul(q1r, q1, rq);
    cq[0] = q1r[0]; cq[1] = -q1r[1]; cq[2] = -q1r[2]; cq[3] = -q1r[3];
    quat_mul(e, cq, q2);
    // the lane's dof: angular motion (cdof's rotational part) of body2 minus body1
    float wv[4] = {0, 0, 0, 0}, de[4] = {0, 0, 0, 0};
    if (lane < nv) {
      const int bj = m.dof_bodyid[lane], be = m.body_subtree_end[bj];
      const bool a1 = o1 >= bj && o1 < be, a2 = o2 >= bj && o2 < be;
      for (int i = 0; i < 3; ++i) wv[1 + i] = (a2 ? s[L.cdof + 6 * lane + i] : 0.0f) - (a1 ? s[L.cdof + 6 * lane + i] : 0.0f);
      float tq[4];
      quat_mul(tq, cq, wv);
      quat_mul(de, tq, q2);
    }
    const float rdiag = m.body_invweight0[2 * o1 + 1] + m.body_invweight0[2 * o2 + 1];
    for (int k = 0; k < 3; ++k) {
      if (lane < nv) J[nefc * nv + lane] = 0.5f * de[1 + k] * ts;
      if (lane == 0) {
        type[nefc] = __int_as_float(code);
        pos[nefc] = e[1 + k] * ts; marg[nefc] = 0; floss[nefc] = kEqBound; bb[nefc] = rdiag;
      }
      ++nefc;
    }
  }
  if (m.neq > 0) wsync();
  // --- friction loss rows
  if (!(m.disableflags & MRS_DSBL_FRICTIONLOSS)) {
    const int r0 = nefc;
    #pragma unroll 1
    for (int k = 0; k < m.nfric; ++k) {
      const int j = m.fric_dof[k], r = r0 + k;
      if (lane < nv) J[r * nv + lane] = (lane == j) ? 1.0f : 0.0f;
      if (lane == 0) {
        type[r] = __int_as_float(EFC_FRICTION * 65536 + j);
        pos[r] = 0; marg[r] = 0; floss[r] = m.dof_frictionloss[j];
      }
    }
    nefc = r0 + m.nfric;
    // tendon friction loss rows, J = ten_J (mj_instantiateFriction: after the dofs')
    #pragma unroll 1
    for (int k = 0; k < m.nten_fric; ++k) {
      const int t = m.ten_fric[k], r = nefc + k;
      if (lane < nv) J[r * nv + lane] = m.ten_J[t * nv + lane];
      if (lane == 0) {
        type[r] = __int_as_float(EFC_TFRICTION * 65536 + t);
        pos[r] = 0; marg[r] = 0; floss[r] = m.ten_prm[12 * t + 7];
      }
    }
    nefc += m.nten_fric;
  }
  // --- joint limit rows (lane per limited joint, compacted)
  if (!(m.disableflags & MRS_DSBL_LIMIT)) {
    const int lim0 = nefc;
    #pragma unroll 1
    for (int base = 0; base < m.nlim; base += G) {
      const int k = base + lane;
      int cnt = 0;
      float dist[2] = {0, 0};
      int jid = -1;
      bool act[2] = {false, false};
      if (k < m.nlim) {
        jid = m.lim_jnt[k];
        const float q = s[L.qpos + m.jnt_qposadr[jid]], mg = m.jnt_margin[jid];
        dist[0] = q - m.jnt_range[2 * jid];
        dist[1] = m.jnt_range[2 * jid + 1] - q;
        act[0] = dist[0] < mg;
        act[1] = dist[1] < mg;
        cnt = (int)act[0] + (int)act[1];
      }
      int total;
      int off = gscan_excl_small<G, 2>(cnt, total);  // (cnt <= 2)
      int r = nefc + off;
      for (int sd = 0; sd < 2; ++sd) {
        if (!act[sd]) continue;
        type[r] = __int_as_float(EFC_LIMIT * 65536 + jid);
        pos[r] = dist[sd];
        marg[r] = m.jnt_margin[jid];
        floss[r] = sd == 0 ? 1.0f : -1.0f;  // J sign, used below
        ++r;
      }
      nefc += total;
    }
    wsync();
    // dense J of limit rows
    #pragma unroll 1
    for (int r = lim0; r < nefc; ++r) {
      const int code = __float_as_int(type[r]);
      const int jid = code & 0xffff;
      const int dof = m.jnt_dofadr[jid];
      const float sg = floss[r];
      if (lane < nv) J[r * nv + lane] = (lane == dof) ? sg : 0.0f;
    }
    wsync();
    if (lane == 0)
      #pragma unroll 1
      for (int r = lim0; r < nefc; ++r) floss[r] = 0;
    // tendon limit rows, lower then upper, J = +-ten_J (mj_instantiateLimit: after the joints')
    #pragma unroll 1
    for (int k = 0; k < m.nten_lim; ++k) {
      const int t = m.ten_lim[k];
      const CPtr<float> tp = m.ten_prm + 12 * t;
      const float len = s[L.ten + 2 * t], mg = tp[6];
      const float dist[2] = {len - tp[4], tp[5] - len};
      for (int sd = 0; sd < 2; ++sd) {
        if (!(dist[sd] < mg)) continue;
        if (lane < nv) J[nefc * nv + lane] = sd == 0 ? m.ten_J[t * nv + lane] : -m.ten_J[t * nv + lane];
        if (lane == 0) {
          type[nefc] = __int_as_float(EFC_TLIMIT * 65536 + t);
          pos[nefc] = dist[sd]; marg[nefc] = mg; floss[nefc] = 0;
        }
        ++nefc;
      }
    }
    if (m.nten_lim > 0) wsync();
  }
  // --- contact rows: lane per dof, loop over contacts
  if constexpr (G == 64) {
    // blocked mode (Newton / CG): every contact's record and pair data are loaded lane-parallel up
    // front (lane = contact) and taken by readlane in the row loop, whose Jacobian columns then come
    // from LDS alone (jac_col_blk) -- no dependent global round trip per contact
    #pragma unroll 1
    for (int c0 = 0; c0 < ncon; c0 += 64) {
      const int ci = c0 + lane;
      const bool in = ci < ncon;
      const gfloat* rc = scr + S.con + kConRec * (in ? ci : c0);
      const int pl = __float_as_int(rc[0]);
      float cv[13];
      for (int i = 0; i < 13; ++i) cv[i] = rc[1 + i];  // dist, pos[3], frame[9]
      const int dl = m.pair_dim[pl];
      const int b1l = m.geom_bodyid[m.pair_g1[pl]], b2l = m.geom_bodyid[m.pair_g2[pl]];
      const int r1l = m.body_rootid[b1l], r2l = m.body_rootid[b2l];
      const float mul = m.pair_friction[3 * pl], mgl = m.pair_margin[pl] - m.pair_gap[pl];
      const int nc = ncon - c0 < 64 ? ncon - c0 : 64;
      #pragma unroll 1
      for (int k = 0; k < nc; ++k) {
        const int c = c0 + k;
        const int dim = __builtin_amdgcn_readlane(dl, k);
        const int b1 = __builtin_amdgcn_readlane(b1l, k), b2 = __builtin_amdgcn_readlane(b2l, k);
        const int r1 = __builtin_amdgcn_readlane(r1l, k), r2 = __builtin_amdgcn_readlane(r2l, k);
        const float dist = bcast(cv[0], k), mu = bcast(mul, k), mg = bcast(mgl, k);
        float cp[3] = {bcast(cv[1], k), bcast(cv[2], k), bcast(cv[3], k)};
        float fr[9];
        for (int i = 0; i < 9; ++i) fr[i] = bcast(cv[4 + i], k);
        const bool ell = dim == 3 && m.cone == MRS_CONE_ELLIPTIC;
        const int nrow = dim == 1 ? 1 : (ell ? 3 : 4);
        if (lane == 0) scr[S.con + kConRec * c + 14] = __int_as_float(nefc + nrow <= m.max_efc ? nefc : -1);
        float jc[3] = {0, 0, 0};
        if (lane < nv) {
          float c1[3], c2[3];
          jac_col_blk(s, L, b1, r1, cp, lane, c1);
          jac_col_blk(s, L, b2, r2, cp, lane, c2);
          const float dc[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
          for (int r = 0; r < 3; ++r) jc[r] = fr[3 * r] * dc[0] + fr[3 * r + 1] * dc[1] + fr[3 * r + 2] * dc[2];
        }
        if (ell && nefc + nrow > m.max_efc) continue;  // (an elliptic block is kept whole)
        for (int q = 0; q < nrow; ++q) {
          if (nefc >= m.max_efc) break;
          // pyramid edges: both tangent directions use the sliding coefficient (mj_setContact);
          // elliptic: the frame rows themselves, k + 1 in the floss slot
          const int kk = 1 + (q >> 1);
          const float sg = (q & 1) ? -1.0f : 1.0f;
          if (lane < nv)
            J[nefc * nv + lane] = (dim == 1 || (ell && q == 0)) ? jc[0]
                                  : (ell ? (q == 1 ? jc[1] : jc[2]) : jc[0] + sg * mu * (kk == 1 ? jc[1] : jc[2]));
          if (lane == 0) {
            type[nefc] = __int_as_float(EFC_CONTACT * 65536 + c);
            pos[nefc] = dist; marg[nefc] = mg; floss[nefc] = ell ? (float)(q + 1) : 0.0f;
          }
          ++nefc;
        }
      }
    }
  } else
  #pragma unroll 1
  for (int c = 0; c < ncon; ++c) {
    gfloat* rec = scr + S.con + kConRec * c;
    const int p = __float_as_int(rec[0]);
    const int dim = m.pair_dim[p];
    const int b1 = m.geom_bodyid[m.pair_g1[p]], b2 = m.geom_bodyid[m.pair_g2[p]];
    float cp[3] = {rec[2], rec[3], rec[4]};
    // first efc row of this contact (rec[14]; -1 if the row cap cut its rows), for cfrc_ext
    const bool ell = dim == 3 && m.cone == MRS_CONE_ELLIPTIC;
    if (lane == 0) rec[14] = __int_as_float(nefc + (dim == 1 ? 1 : (ell ? 3 : 4)) <= m.max_efc ? nefc : -1);
    float jc[3] = {0, 0, 0};
    if (lane < nv) {
      float c1[3], c2[3];
      jac_col(m, s, b1, cp, lane, c1);
      jac_col(m, s, b2, cp, lane, c2);
      float dc[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
      for (int r = 0; r < 3; ++r) jc[r] = rec[5 + 3 * r] * dc[0] + rec[6 + 3 * r] * dc[1] + rec[7 + 3 * r] * dc[2];
    }
    if (ell) {
      // elliptic cone: the frame rows (normal, tangent 1, tangent 2), kept whole, k + 1 in floss
      if (nefc + 3 <= m.max_efc)
        for (int k = 0; k < 3; ++k) {
          if (lane < nv) J[nefc * nv + lane] = jc[k];
          if (lane == 0) {
            type[nefc] = __int_as_float(EFC_CONTACT * 65536 + c);
            pos[nefc] = rec[1]; marg[nefc] = m.pair_margin[p] - m.pair_gap[p]; floss[nefc] = (float)(k + 1);
          }
          ++nefc;
        }
    } else if (dim == 1) {
      if (nefc < m.max_efc) {
        if (lane < nv) J[nefc * nv + lane] = jc[0];
        if (lane == 0) {
          type[nefc] = __int_as_float(EFC_CONTACT * 65536 + c);
          pos[nefc] = rec[1]; marg[nefc] = m.pair_margin[p] - m.pair_gap[p]; floss[nefc] = 0;
        }
        ++nefc;
      }
    } else {
      for (int k = 1; k < 3; ++k)
        for (int sg = 1; sg >= -1; sg -= 2) {
          if (nefc >= m.max_efc) continue;
          // both tangent directions use the sliding coefficient (contact friction is
          // (slide, slide, spin, roll, roll) from the geoms' (slide, spin, roll), mj_setContact)
          const float mu = m.pair_friction[3 * p];
          if (lane < nv) J[nefc * nv + lane] = jc[0] + sg * mu * jc[k];
          if (lane == 0) {
            type[nefc] = __int_as_float(EFC_CONTACT * 65536 + c);
            pos[nefc] = rec[1]; marg[nefc] = m.pair_margin[p] - m.pair_gap[p]; floss[nefc] = 0;
          }
          ++nefc;
        }
    }
  }
  if (lane == 0) scr[S.efc_n] = __int_as_float(nefc);
  wsync();
  return nefc;
}

template <int G, bool kPrimal, bool kHot>
__device__ float constraints_dense(ENV_PARAMS, int ncon, float qacc_s, int pre_nefc) {
  ENV_UNPACK;
  if constexpr (G == 64) ncon = uniform_int(ncon);
  const int nv = m.nv;
  gfloat* J = scr + S.efc_J;
  gfloat* MJ = scr + S.efc_MJ;
  gfloat* type = scr + S.efc_type;
  gfloat* pos = scr + S.efc_pos;
  gfloat* marg = scr + S.efc_margin;
  gfloat* floss = scr + S.efc_floss;
  gfloat* Rr = scr + S.efc_R;
  gfloat* aref = scr + S.efc_aref;
  gfloat* bb = scr + S.efc_b;
  gfloat* ff = scr + S.efc_f;
  gfloat* ARii = scr + S.efc_ARii;
  unsigned long long t_sub = SUB_T();
  // the rows (pre_nefc >= 0: already built by the workgroup's helper wave, step_kernel)
  const int nefc = pre_nefc >= 0 ? pre_nefc : dense_rows<G>(ENV_ARGS, ncon);
  SUB_ADD(PH_CON_ROWS, t_sub);
  t_sub = SUB_T();
  if (nefc == 0) {
    if (lane < nv) s[L.qfrc_con + lane] = 0;
    wsync();
    return qacc_s;
  }
  // --- impedance, R, aref, M^-1 J', ARii, b (lane per row); the primal solvers need R and aref only
  // (kPrimal: the kernel instantiated for Newton / CG models, so the dual PGS paths below are not
  // compiled into it)
  const bool primal = kPrimal || m.solver != MRS_SOL_PGS;
  // register-resident solvers (dual PGS or primal) for small systems; elliptic blocks take the
  // generic paths below
  const bool small = G == 16 && nefc <= 16 && !(m.cone == MRS_CONE_ELLIPTIC && ncon > 0);
  float my_R = 1, my_aref = 0, my_b = 0, my_fl = 0;
  bool my_fric = false;
  #pragma unroll 1
  for (int r = lane; r < nefc; r += G) {
    const int code = __float_as_int(type[r]);
    const int t = code >> 16;
    // R and aref (mj_makeImpedance), from the helper wave when it built the rows
    float R, ar;
    if (pre_nefc >= 0) {
      R = Rr[r];
      ar = aref[r];
    } else {
      row_impedance<G>(m, s, scr, r, R, ar);
      Rr[r] = R;
    }
    float jqs = 0;
    const gfloat* Jr = J + r * nv;
    #pragma unroll 4
    for (int j = 0; j < nv; ++j) jqs += Jr[j] * s[L.qacc_smooth + j];
    if (small) {
      my_R = R;
      my_aref = ar;
      my_b = jqs - my_aref;
      my_fl = fric_like(t) ? floss[r] : 0.0f;
      my_fric = fric_like(t);
      aref[r] = my_aref;
      continue;
    }
    aref[r] = ar;
    bb[r] = jqs - aref[r];
    if (primal || G == 64) continue;
    // M^-1 J_r'
    gfloat* MJr = MJ + r * nv;
    chol_solve_serial(s + L.L, nv, Jr, MJr);
    float d = 0;
    #pragma unroll 1
    for (int j = 0; j < nv; ++j) d += Jr[j] * MJr[j];
    ARii[r] = d + R;
  }
  wsync();
  if constexpr (G == 64) {
    // blocked mode (elliptic PGS): L.L holds the per-tree block factor, so M^-1 J_r' is the
    // wave's lane-per-dof block solve, one row at a time
    if (!primal) {
      #pragma unroll 1
      for (int r = 0; r < nefc; ++r) {
        const float jr = lane < nv ? J[r * nv + lane] : 0.0f;
        float y;
        MRS_CALL(G, y = chol_solve_lanes<G>(mp, s + L.L, jr, lane));
        if (lane < nv) MJ[r * nv + lane] = y;
        const float d = gsum<G>(lane < nv ? jr * y : 0.0f);
        if (lane == 0) ARii[r] = d + Rr[r];
      }
      wsync();
    }
  }
  SUB_ADD(PH_CON_REC, t_sub);
  t_sub = SUB_T();
  int rmax = 0;
  if constexpr (G == 16) {
    // rows unrolled up to the largest small system among the wave's active groups (wave-uniform
    // bound; binary search with ballots, which only see active lanes)
    const int mine = small ? nefc : 0;
#pragma unroll
    for (int bit = 16; bit >= 1; bit >>= 1)
      if (__ballot(mine >= rmax + bit) != 0) rmax += bit;
  }
  if (primal) {
    float qa;
    const bool newton = m.solver == MRS_SOL_NEWTON;
    if constexpr (G == 16 && kPrimal) {  // (the G = 16 kernel instantiated for Newton / CG models)
      if (small) {
        auto solve = [&](auto kv) {
          constexpr int KV = decltype(kv)::value;
          if (rmax <= 4) return primal_small16<false, 4, KV>(ENV_ARGS, J, ff, nefc, my_R, my_aref, my_fl, my_fric, qacc_s, newton);
          if (rmax <= 8) return primal_small16<false, 8, KV>(ENV_ARGS, J, ff, nefc, my_R, my_aref, my_fl, my_fric, qacc_s, newton);
          return primal_small16<false, 16, KV>(ENV_ARGS, J, ff, nefc, my_R, my_aref, my_fl, my_fric, qacc_s, newton);
        };
        qa = nv <= 8 ? solve(std::integral_constant<int, 8>{}) : solve(std::integral_constant<int, 16>{});
        SUB_ADD(PH_CON_PGS, t_sub);
        return qa;
      }
    }
    [[clang::noinline]] qa = solve_primal<G>(ENV_ARGS, nefc, newton);
    SUB_ADD(PH_CON_PGS, t_sub);
    return qa;
  }
  if constexpr (G == 16) {
    if (small) {
      // rows unrolled to the wave's row count, the substitutions to the model's dof count (nv can
      // exceed the row count: a free body with one contact, an arm with one active limit)
      auto solve = [&](auto kv) {
        constexpr int KV = decltype(kv)::value;
        if (rmax <= 4) return pgs_small16<false, 4, KV, kHot>(m, s, J, ff, nefc, rmax, my_R, my_aref, my_b, my_fl, qacc_s, lane);
        if (rmax <= 8) return pgs_small16<false, 8, KV, kHot>(m, s, J, ff, nefc, rmax, my_R, my_aref, my_b, my_fl, qacc_s, lane);
        if (rmax <= 12) return pgs_small16<false, 12, KV, kHot>(m, s, J, ff, nefc, rmax, my_R, my_aref, my_b, my_fl, qacc_s, lane);
        return pgs_small16<false, 16, KV, kHot>(m, s, J, ff, nefc, rmax, my_R, my_aref, my_b, my_fl, qacc_s, lane);
      };
      float qa = nv <= 8 ? solve(std::integral_constant<int, 8>{}) : solve(std::integral_constant<int, 16>{});
      wsync();
      SUB_ADD(PH_CON_PGS, t_sub);
      return qa;
    }
  }
  // --- warm start: forces of mj_constraintUpdate at qacc_warmstart, kept if dual cost < 0
  float qa = lane < nv ? qacc_s : 0.0f;  // qacc = qacc_smooth + M^-1 J' f, lane per dof
  {
    bool warm = !(m.disableflags & MRS_DSBL_WARMSTART);
    #pragma unroll 1
    for (int r = lane; r < nefc; r += G) {
      float f = 0;
      if (m.cone == MRS_CONE_ELLIPTIC && (__float_as_int(type[r]) >> 16) == EFC_CONTACT && floss[r] > 0.5f) {
        // elliptic block: its first row's lane writes the three forces (the zone forces of
        // mj_constraintUpdate at qacc_warmstart)
        if (floss[r] != 1.0f) continue;
        float f3[3] = {0, 0, 0};
        if (warm) {
          float jar3[3], D[3];
          for (int k = 0; k < 3; ++k) {
            const gfloat* Jr = J + (r + k) * nv;
            float jar = -aref[r + k];
            #pragma unroll 1
            for (int j = 0; j < nv; ++j) jar += Jr[j] * s[L.qacc_ws + j];
            jar3[k] = jar;
            D[k] = 1.0f / Rr[r + k];
          }
          ell_zone(ell_friction(m, scr, type, r), m.impratio, D, jar3, f3, nullptr, nullptr);
        }
        for (int k = 0; k < 3; ++k) ff[r + k] = f3[k];
        continue;
      }
      if (warm) {
        const gfloat* Jr = J + r * nv;
        float jar = -aref[r];
        #pragma unroll 1
        for (int j = 0; j < nv; ++j) jar += Jr[j] * s[L.qacc_ws + j];
        const int t = __float_as_int(type[r]) >> 16;
        const float D = 1.0f / Rr[r];
        if (fric_like(t)) {
          const float fl = floss[r];
          f = jar <= -Rr[r] * fl ? fl : (jar >= Rr[r] * fl ? -fl : -D * jar);
        } else {
          f = jar < 0 ? -D * jar : 0.0f;
        }
      }
      ff[r] = f;
    }
    wsync();
    if (warm) {
      // v = M^-1 J' f (lane per dof); cost = sum_r f_r (0.5 (J_r v + R_r f_r) + b_r)
      float v = 0;
      if (lane < nv)
        #pragma unroll 1
        for (int r = 0; r < nefc; ++r) v += MJ[r * nv + lane] * ff[r];
      float cost = 0;
      #pragma unroll 1
      for (int r = 0; r < nefc; ++r) {
        const float jv = gsum<G>(lane < nv ? J[r * nv + lane] * v : 0.0f);
        cost += ff[r] * (0.5f * (jv + Rr[r] * ff[r]) + bb[r]);
      }
      if (cost > 0) {
        #pragma unroll 1
        for (int r = lane; r < nefc; r += G) ff[r] = 0;
      } else {
        qa += v;
      }
      wsync();
    }
  }
  // --- PGS sweeps (rows serial, dot products across lanes)
  int nit = 0;  // sweeps done (mjData.solver_niter)
  if (m.cone == MRS_CONE_ELLIPTIC) {
    // elliptic models: the sweeps keep qacc, the residuals and the row forces in fp64 (the split block
    // update's slow convergence carries fp32 rounding of its iterate into the result, qcqp2_la); the
    // solver's inputs (J, M^-1 J', the Delassus entries, aref, R) stay the fp32 ones built above
    typedef __attribute__((address_space(1))) double gdouble;
    gdouble* fd = (gdouble*)(scr + S.efc_fd);
    #pragma unroll 1
    for (int r = lane; r < nefc; r += G) fd[r] = ff[r];
    wsync();
    double qd = lane < nv ? static_cast<double>(qa) : 0.0;
    #pragma unroll 1
    for (int it = 0; it < m.iterations; ++it) {
      double improvement = 0;
      #pragma unroll 1
      for (int r = 0; r < nefc; ++r) {
        if (ell_start(m, type, floss, r)) {
          // elliptic block: mj_solPGS's split update (ell_pgs_split), or with the opt-in
          // MRS_RESTATE_PGS_ELLIPTIC_BLOCK the exact minimiser of the block's local cost over the cone
          // (ell_block_min; oracle.c fwd_constraint)
          double res[3], A[9], old[3], c[3], y[3];
          for (int k = 0; k < 3; ++k) {
            old[k] = fd[r + k];
            res[k] = gsum_d<G>(lane < nv ? static_cast<double>(J[(r + k) * nv + lane]) * qd : 0.0) - aref[r + k] +
                     static_cast<double>(Rr[r + k]) * old[k];
            A[4 * k] = ARii[r + k];
          }
          for (int a = 0; a < 3; ++a)
            for (int b = a + 1; b < 3; ++b)
              A[3 * a + b] = A[3 * b + a] = gsum<G>(lane < nv ? J[(r + a) * nv + lane] * MJ[(r + b) * nv + lane] : 0.0f);
          for (int k = 0; k < 3; ++k) c[k] = res[k] - (A[3 * k] * old[0] + A[3 * k + 1] * old[1] + A[3 * k + 2] * old[2]);
          if (m.restate & MRS_RESTATE_PGS_ELLIPTIC_BLOCK) ell_block_min(A, c, ell_friction(m, scr, type, r), y);
          else ell_pgs_split(A, res, old, ell_friction(m, scr, type, r), y);
          double dl[3], quad = 0;
          for (int k = 0; k < 3; ++k) dl[k] = y[k] - old[k];
          for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) quad += dl[a] * A[3 * a + b] * dl[b];
          if (lane < nv)
            qd += static_cast<double>(MJ[r * nv + lane]) * dl[0] + static_cast<double>(MJ[(r + 1) * nv + lane]) * dl[1] +
                  static_cast<double>(MJ[(r + 2) * nv + lane]) * dl[2];
          if (lane == 0) { fd[r] = y[0]; fd[r + 1] = y[1]; fd[r + 2] = y[2]; }
          improvement -= dl[0] * res[0] + dl[1] * res[1] + dl[2] * res[2] + 0.5 * quad;
          wsync();
          r += 2;
          continue;
        }
        const double jq = gsum_d<G>(lane < nv ? static_cast<double>(J[r * nv + lane]) * qd : 0.0);
        const double f0 = fd[r];
        const double res = jq - aref[r] + static_cast<double>(Rr[r]) * f0;
        const double a = ARii[r];
        double nf = f0 - res / a;
        const int t = __float_as_int(type[r]) >> 16;
        if (fric_like(t)) nf = fmin(fmax(nf, -static_cast<double>(floss[r])), static_cast<double>(floss[r]));
        else if (nf < 0) nf = 0;
        const double delta = nf - f0;
        if (delta != 0) {
          if (lane < nv) qd += static_cast<double>(MJ[r * nv + lane]) * delta;
          if (lane == 0) fd[r] = nf;
        }
        improvement -= delta * res + 0.5 * delta * delta * a;
        wsync();
      }
      nit = it + 1;
      if (improvement * m.pgs_scale < m.tolerance) break;
    }
    if (lane == 0) s[L.niter] = __int_as_float(nit);
    // qfrc_constraint = J' f; the row forces exported in fp32 (mrs_batch_get_efc)
    if (lane < nv) {
      double v = 0;
      #pragma unroll 1
      for (int r = 0; r < nefc; ++r) v += static_cast<double>(J[r * nv + lane]) * fd[r];
      s[L.qfrc_con + lane] = static_cast<float>(v);
    }
    #pragma unroll 1
    for (int r = lane; r < nefc; r += G) ff[r] = static_cast<float>(fd[r]);
    wsync();
    return static_cast<float>(qd);
  }
  #pragma unroll 1
  for (int it = 0; it < m.iterations; ++it) {
    float improvement = 0;
    #pragma unroll 1
    for (int r = 0; r < nefc; ++r) {
      const float jq = gsum<G>(lane < nv ? J[r * nv + lane] * qa : 0.0f);
      const float f0 = ff[r];
      const float res = jq - aref[r] + Rr[r] * f0;
      const float a = ARii[r];
      float nf = f0 - res / a;
      const int t = __float_as_int(type[r]) >> 16;
      if (fric_like(t)) nf = clampf(nf, -floss[r], floss[r]);
      else if (nf < 0) nf = 0;
      const float delta = nf - f0;
      if (delta != 0) {
        if (lane < nv) qa += MJ[r * nv + lane] * delta;
        if (lane == 0) ff[r] = nf;
      }
      improvement -= delta * res + 0.5f * delta * delta * a;
      wsync();
    }
    nit = it + 1;
    if (improvement * m.pgs_scale < m.tolerance) break;
  }
  if (lane == 0) s[L.niter] = __int_as_float(nit);
  // --- qfrc_constraint = J' f
  if (lane < nv) {
    float v = 0;
    #pragma unroll 1
    for (int r = 0; r < nefc; ++r) v += J[r * nv + lane] * ff[r];
    s[L.qfrc_con + lane] = v;
  }
  wsync();
  return qa;
}

// mj_rnePostConstraint (models with accelerometer / force / torque sensors only): cacc including qacc
// (world: -gravity) into L.cacc; cfrc_ext from the contact forces (pyramid rows decoded to one world
// force per row, applied at the contact point, moved to the subtree com; body2 +, body1 -);
// cfrc_int = cinert cacc + cvel x* (cinert cvel) - cfrc_ext into L.cfrc, summed over subtrees into
// L.crb.  Needs L.qacc and the row forces (efc_f) of this step.
template <int G>
__device__ MRS_PHASE void rne_post(ENV_PARAMS, int ncon) {
  ENV_UNPACK;
  float g0[6] = {0, 0, 0, 0, 0, 0};
  if (!(m.disableflags & MRS_DSBL_GRAVITY)) { g0[3] = -m.gravity[0]; g0[4] = -m.gravity[1]; g0[5] = -m.gravity[2]; }
  auto own = [&](int b, float v[6]) {
    const int da = m.body_dofadr[b], nd = m.body_dofnum[b];
    for (int j = da; j < da + nd; ++j) {
      const float qv = s[L.qvel + j], qa = s[L.qacc + j];
      for (int i = 0; i < 6; ++i) v[i] += s[L.cdofdot + 6 * j + i] * qv + s[L.cdof + 6 * j + i] * qa;
    }
  };
  if (m.nbody <= G) {
    const int b = lane;
    float v[6] = {0, 0, 0, 0, 0, 0};
    if (b >= 1 && b < m.nbody) own(b, v);
    tree_prefix6<G>(m, s + L.cacc, b, v);
    if (b < m.nbody)
      for (int i = 0; i < 6; ++i) s[L.cacc + 6 * b + i] = v[i] + g0[i];
    wsync();
  } else {
    if (lane < 6) s[L.cacc + lane] = g0[lane];
    wsync();
    for (int lev = 1; lev <= m.max_depth; ++lev) {
      const int a0 = m.level_adr[lev], nl = m.level_num[lev];
      #pragma unroll 1
      for (int k = lane; k < nl; k += G) {
        const int b = m.level_body[a0 + k];
        float v[6];
        for (int i = 0; i < 6; ++i) v[i] = s[L.cacc + 6 * m.body_parentid[b] + i];
        own(b, v);
        for (int i = 0; i < 6; ++i) s[L.cacc + 6 * b + i] = v[i];
      }
      wsync();
    }
  }
  const gfloat* ff = scr + S.efc_f;
  #pragma unroll 1
  for (int b = lane; b < m.nbody; b += G) {
    float fi[6] = {0, 0, 0, 0, 0, 0};
    if (b != 0) {
      float ca[6], cv[6], f1[6], t[6], f2[6];
      for (int i = 0; i < 6; ++i) { ca[i] = s[L.cacc + 6 * b + i]; cv[i] = s[L.cvel + 6 * b + i]; }
      mul_inert_vec(f1, s + L.cinert + 10 * b, ca);
      mul_inert_vec(t, s + L.cinert + 10 * b, cv);
      cross_force(f2, cv, t);
      for (int i = 0; i < 6; ++i) fi[i] = f1[i] + f2[i];
      const int rt = m.body_rootid[b];
      const float c3[3] = {s[L.scom + 3 * rt], s[L.scom + 3 * rt + 1], s[L.scom + 3 * rt + 2]};
      #pragma unroll 1
      for (int c = 0; c < ncon; ++c) {
        const gfloat* rec = scr + S.con + kConRec * c;
        const int p = __float_as_int(rec[0]);
        const int b1 = m.geom_bodyid[m.pair_g1[p]], b2 = m.geom_bodyid[m.pair_g2[p]];
        const int r0 = __float_as_int(rec[14]);
        if ((b != b1 && b != b2) || r0 < 0) continue;
        // contact-frame force (mju_decodePyramid), then world: frame' lfrc
        float lf[3] = {0, 0, 0};
        if (m.pair_dim[p] == 1) {
          lf[0] = ff[r0];
        } else if (m.cone == MRS_CONE_ELLIPTIC) {
          for (int i = 0; i < 3; ++i) lf[i] = ff[r0 + i];  // (normal, tangent 1, tangent 2)
        } else {
          for (int k = 0; k < 2; ++k) {
            const float fp = ff[r0 + 2 * k], fm = ff[r0 + 2 * k + 1];
            lf[0] += fp + fm;
            lf[k + 1] = (fp - fm) * m.pair_friction[3 * p];
          }
        }
        float F[3];
        for (int i = 0; i < 3; ++i) F[i] = rec[5 + i] * lf[0] + rec[8 + i] * lf[1] + rec[11 + i] * lf[2];
        const float d[3] = {rec[2] - c3[0], rec[3] - c3[1], rec[4] - c3[2]};
        float tq[3];
        cross3(tq, d, F);  // torque about the subtree com: (pos - com) x F
        const float sg = b == b2 ? -1.0f : 1.0f;  // cfrc_int subtracts cfrc_ext (+ for body2)
        for (int i = 0; i < 3; ++i) { fi[i] += sg * tq[i]; fi[3 + i] += sg * F[i]; }
      }
    }
    for (int i = 0; i < 6; ++i) s[L.cfrc + 6 * b + i] = fi[i];
  }
  wsync();
  #pragma unroll 1
  for (int b = lane; b < m.nbody; b += G) {
    float acc[6] = {0, 0, 0, 0, 0, 0};
    const int e = b == 0 ? m.nbody : m.body_subtree_end[b];  // the world's subtree is everything
    #pragma unroll 4
    for (int k = b; k < e; ++k)
      for (int i = 0; i < 6; ++i) acc[i] += s[L.cfrc + 6 * k + i];
    for (int i = 0; i < 6; ++i) s[L.crb + 6 * b + i] = acc[i];
  }
  wsync();
}

// rays per lane per pass over the geoms: 4 with lane groups (measured C3: 1.59 ms per launch vs
// 1.98 at 1, 1.71 at 2), 2 at one env per wave (64-VGPR budget: 2.15 ms vs 2.38 at 1, 2.95 at 4)
template <int G>
struct RayBatch { static constexpr int value = G == 64 ? 2 : 4; };
#ifdef MRS_DIAG_SENS_LAST
#define MRS_SD_OK(p) ((p) != nullptr)
#else
#define MRS_SD_OK(p) true
#endif

// R rangefinders per lane in one pass over the geoms (mj_ray per sensor: nearest hit along the
// site's +z over all visible geoms not on the site's body).  Each geom's pose is read from LDS once
// for the R rays, and the R independent rays give the scheduler parallel work.  Rays k0 + j*stride.
// kChunk: the pass covers ray geoms goff .. goff + 31 of a model with more than 32 (rays_chunked);
// otherwise goff is 0 and the code is the <= 32-geom pass
template <int G, int R, bool kChunk = false>
__device__ __forceinline__ void rangefinders(const DevModel& m, const lfloat* se, gfloat* sd, int k0, int stride,
                                             unsigned gmask, int common_body, const float* common_o, int goff_ = 0) {
  const int goff = kChunk ? goff_ : 0;
  const LdsLayout& L = m.L;
  float pnt[R][3], vec[R][3], dist[R];
  int bod[R], adr[R];
  bool act[R];
  unsigned long long t_setup = SUB_T();
  if (common_body >= 0) {
    // every ray of the pass starts at the same point of the same body: one rotation for all (none
    // for a static lidar, whose rays are stored in the world frame)
    const int b = common_body;
    float bm[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, o[3] = {common_o[0], common_o[1], common_o[2]};
    if (!m.rf_static_frame) {
      float bq[4] = {se[L.xquat + 4 * b], se[L.xquat + 4 * b + 1], se[L.xquat + 4 * b + 2], se[L.xquat + 4 * b + 3]};
      quat2mat(bm, bq);
      mat_vec(o, bm, common_o);
      for (int i = 0; i < 3; ++i) o[i] += se[L.xpos + 3 * b + i];
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int k = k0 + j * stride;
      act[j] = k < m.nrf;
      // the ray table is staged in workgroup LDS only when every ray shares body and origin
      // (rf_common); a pass that shares them in a model that does not reads the model block
      float dl[3];
      if (m.rf_common) {
        const lfloat* rr = shared_lds(m) + m.shr_rf + 4 * (act[j] ? k : 0);
        dl[0] = rr[0]; dl[1] = rr[1]; dl[2] = rr[2];
        adr[j] = __float_as_int(rr[3]);
      } else {
        const CPtr<float> rr = m.rfray + 8 * (act[j] ? k : 0);
        dl[0] = rr[0]; dl[1] = rr[1]; dl[2] = rr[2];
        adr[j] = __float_as_int(rr[3]);
      }
      bod[j] = b;
      if (m.rf_static_frame) { vec[j][0] = dl[0]; vec[j][1] = dl[1]; vec[j][2] = dl[2]; }
      else mat_vec(vec[j], bm, dl);
      for (int i = 0; i < 3; ++i) pnt[j][i] = o[i];
      // static split: start from the ray's hit on the world-welded geoms (never beaten: -1); later
      // chunks of ray geoms start from the earlier chunks' nearest hit in the output slot
      dist[j] = m.rf_mode == 2 ? (float)shared_lds(m)[m.shr_rfst + (act[j] ? k : 0)] : -1.0f;
      if (kChunk && goff > 0) dist[j] = act[j] && MRS_SD_OK(sd) ? (float)sd[adr[j]] : -1.0f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int k = k0 + j * stride;
      act[j] = k < m.nrf;
      const CPtr<float> rr = m.rfray + 8 * (act[j] ? k : 0);
      const float dl[3] = {rr[0], rr[1], rr[2]}, ol[3] = {rr[5], rr[6], rr[7]};
      adr[j] = __float_as_int(rr[3]);
      const int b = __float_as_int(rr[4]);
      bod[j] = b;
      if (m.rf_static_frame) {
        for (int i = 0; i < 3; ++i) { pnt[j][i] = ol[i]; vec[j][i] = dl[i]; }
      } else {
        float bq[4] = {se[L.xquat + 4 * b], se[L.xquat + 4 * b + 1], se[L.xquat + 4 * b + 2], se[L.xquat + 4 * b + 3]};
        float bm[9];
        quat2mat(bm, bq);
        mat_vec(pnt[j], bm, ol);
        for (int i = 0; i < 3; ++i) pnt[j][i] += se[L.xpos + 3 * b + i];
        mat_vec(vec[j], bm, dl);
      }
      dist[j] = m.rf_mode == 2 ? (float)shared_lds(m)[m.shr_rfst + (act[j] ? k : 0)] : -1.0f;
      if (kChunk && goff > 0) dist[j] = act[j] && MRS_SD_OK(sd) ? (float)sd[adr[j]] : -1.0f;
    }
  }
  SUB_ADD(PH_SENS_SETUP, t_setup);
  unsigned long long t_geoms = SUB_T();
  // geoms some group of the wave still needs (union of the groups' level-1 masks), in order
#if defined(MRS_DIAG_RAYS) && MRS_DIAG_RAYS == 1
  gmask = 0;  // diagnostic build: setup and stores only
#endif
  unsigned wmask = gmask;
  if constexpr (G < 64) {
#pragma unroll
    for (int i = 0; i < 64 / G; ++i) wmask |= __builtin_amdgcn_readlane(gmask, i * G);
  }
  wmask = __builtin_amdgcn_readfirstlane(wmask);
  constexpr int kMaxSlots = 64 / R;
  unsigned long long mneed = 0;  // bit slot * R + j: ray j is a candidate of the slot-th mesh geom
  // chunk-local ray-geom indices of the recorded mesh geoms, and of the rest; slots are taken in
  // ascending index order, so slot s is the s-th set bit of mslot
  unsigned mslot = 0, mover = 0;
  int nms = 0;
  #pragma unroll 1
  while (wmask) {
    const int i = __builtin_ctz(wmask);
    wmask &= wmask - 1;
    const bool gsel = (gmask >> i) & 1u;
    const CPtr<float> rec = m.rgeom + 8 * (goff + i);
    const int g = __float_as_int(rec[0]), type = __float_as_int(rec[1]), gb = __float_as_int(rec[2]);
    const float rb = rec[3] * 1.0001f + 1e-6f;
    const float gp[3] = {se[L.gxpos + 3 * g], se[L.gxpos + 3 * g + 1], se[L.gxpos + 3 * g + 2]};
    // bounding-sphere cull (conservative, branch-free): closest approach of the ray line to the
    // geom centre within rb, centre not behind the origin by more than rb, and no chance of beating
    // the current nearest hit; ray directions are unit (rotation-matrix columns)
    unsigned cmask = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const float dv[3] = {pnt[j][0] - gp[0], pnt[j][1] - gp[1], pnt[j][2] - gp[2]};
      const float tp = -dot3(dv, vec[j]);
      const float d2 = dot3(dv, dv) - tp * tp;
      const bool near = (d2 <= rb * rb) & (tp >= -rb) & ((dist[j] < 0) | (tp - rb <= dist[j]));
      const bool c = gsel & act[j] & (gb != bod[j]) & ((type == MRS_GEOM_PLANE) | near);
      cmask |= static_cast<unsigned>(c) << j;
    }
    if (!__any(cmask != 0)) continue;
    if (type == MRS_GEOM_MESH) {
      // meshes are walked after the pass (below), when the pass's ray arrays are dead: record the
      // candidates (slot of R bits), or walk every ray past MaxSlots mesh geoms
      if (nms < kMaxSlots) {
        mneed |= static_cast<unsigned long long>(cmask) << (nms * R);
        mslot |= 1u << i;
        ++nms;
      } else {
        mover |= 1u << i;
      }
      continue;
    }
    float gm[9];
    for (int k = 0; k < 9; ++k) gm[k] = se[L.gxmat + 9 * g + k];
    const CPtr<float> gs = rec + 4;
    // rays of a pass from one origin: the origin goes into the geom frame once, not once per ray
    float lp0[3] = {0, 0, 0};
    if (common_body >= 0) {
      const float dv[3] = {pnt[0][0] - gp[0], pnt[0][1] - gp[1], pnt[0][2] - gp[2]};
      matT_vec(lp0, gm, dv);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (!((cmask >> j) & 1)) continue;
      float lp[3] = {lp0[0], lp0[1], lp0[2]}, lv[3];
      if (common_body < 0) {
        const float dv[3] = {pnt[j][0] - gp[0], pnt[j][1] - gp[1], pnt[j][2] - gp[2]};
        matT_vec(lp, gm, dv);
      }
      matT_vec(lv, gm, vec[j]);
      float t;
      t = ray_geom_local(type, gs, lp, lv);  // (meshes: the compacted walk above)
      if (t >= 0 && (dist[j] < 0 || t < dist[j])) dist[j] = t;
    }
  }
  if (mslot | mover) {
    // mesh walks.  Each round every lane walks its next candidate (mesh slot, ray j) -- lowest bit of
    // its own record, whichever mesh that is -- so the wave runs max-over-lanes(candidates) walks
    // rather than one per (mesh, ray slot) any lane needs; geoms past kMaxSlots are walked one at a
    // time with every ray.  The ray is rebuilt from the table (the pass's pnt / vec arrays are dead
    // here, which keeps the walk out of their registers)
    auto ray_of = [&](int k, float p[3], float v[3]) {
      int rb;
      if (common_body >= 0) {
        rb = common_body;
        float dl[3];
        if (m.rf_common) {
          const lfloat* rr = shared_lds(m) + m.shr_rf + 4 * k;
          dl[0] = rr[0]; dl[1] = rr[1]; dl[2] = rr[2];
        } else {
          const CPtr<float> rr = m.rfray + 8 * k;
          dl[0] = rr[0]; dl[1] = rr[1]; dl[2] = rr[2];
        }
        p[0] = common_o[0]; p[1] = common_o[1]; p[2] = common_o[2];
        if (m.rf_static_frame) {
          v[0] = dl[0]; v[1] = dl[1]; v[2] = dl[2];
        } else {
          float bq[4] = {se[L.xquat + 4 * rb], se[L.xquat + 4 * rb + 1], se[L.xquat + 4 * rb + 2], se[L.xquat + 4 * rb + 3]};
          float bm[9];
          quat2mat(bm, bq);
          mat_vec(v, bm, dl);
          mat_vec(p, bm, common_o);
          for (int q = 0; q < 3; ++q) p[q] += se[L.xpos + 3 * rb + q];
        }
      } else {
        const CPtr<float> rr = m.rfray + 8 * k;
        const float dl[3] = {rr[0], rr[1], rr[2]}, ol[3] = {rr[5], rr[6], rr[7]};
        rb = __float_as_int(rr[4]);
        if (m.rf_static_frame) {
          for (int q = 0; q < 3; ++q) { p[q] = ol[q]; v[q] = dl[q]; }
        } else {
          float bq[4] = {se[L.xquat + 4 * rb], se[L.xquat + 4 * rb + 1], se[L.xquat + 4 * rb + 2], se[L.xquat + 4 * rb + 3]};
          float bm[9];
          quat2mat(bm, bq);
          mat_vec(p, bm, ol);
          for (int q = 0; q < 3; ++q) p[q] += se[L.xpos + 3 * rb + q];
          mat_vec(v, bm, dl);
        }
      }
      return rb;
    };
    // the pass's results go to their output slots first (sensordata, or the static-hit table in the
    // producer pass); each walk then reads its ray's nearest hit so far from there as the walk's
    // bound and writes a nearer hit back -- the R results leave the registers for the walks
    auto out_of = [&](int k) -> gfloat* {
      if (m.rf_mode == 1) return (gfloat*)(m.rf_static + k);
      const int a = m.rf_common ? __float_as_int(shared_lds(m)[m.shr_rf + 4 * k + 3]) : __float_as_int(m.rfray[8 * k + 3]);
      return sd + a;
    };
    const bool sd_ok = m.rf_mode == 1 || MRS_SD_OK(sd);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (m.rf_mode == 1) {
        if (act[j]) m.rf_static[k0 + j * stride] = dist[j];
      } else if (act[j] && sd_ok) {
        sd[adr[j]] = dist[j];
      }
    }
    // one walk: ray js of this lane against ray geom i (lane-varying)
    auto walk = [&](bool has, int i, int js) {
      const int k = k0 + js * stride;
      float p[3], v[3];
      const int rb = ray_of(k, p, v);
      const CPtr<float> rec = m.rgeom + 8 * (goff + i);
      const int g = __float_as_int(rec[0]), gb = __float_as_int(rec[2]), id = __float_as_int(rec[7]);
      if (has && rb != gb && sd_ok) {
        gfloat* o = out_of(k);
        const float dcur = *o;
        const float dv[3] = {p[0] - se[L.gxpos + 3 * g], p[1] - se[L.gxpos + 3 * g + 1], p[2] - se[L.gxpos + 3 * g + 2]};
        float gm[9], lp[3], lv[3];
        for (int q = 0; q < 9; ++q) gm[q] = se[L.gxmat + 9 * g + q];
        matT_vec(lp, gm, dv);
        matT_vec(lv, gm, v);
        const float t = ray_mesh(m.mesh_tri + 9 * m.mesh_faceadr[id], m.mesh_facenum[id], rec + 4, lp, lv,
                                 m.mesh_bvh + 8 * m.mesh_bvhadr[id], m.mesh_bvhnum[id], nullptr, dcur);
        // (t is dcur itself when the walk found nothing nearer)
        if (t >= 0 && (dcur < 0 || t < dcur)) *o = t;
      }
    };
    unsigned long long need = mneed;
    #pragma unroll 1
    while (__any(need != 0)) {
      const bool has = need != 0;
      const int bit = has ? __builtin_ctzll(need) : 0;
      need &= need - 1;
      const int sl = bit / R;
      unsigned ms = mslot;  // the sl-th set bit of mslot: slot sl's ray geom
      #pragma unroll 1
      for (int q = 0; q < sl; ++q) ms &= ms - 1;
      walk(has, __builtin_ctz(ms | 0x80000000u), bit - sl * R);
    }
    unsigned actm = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) actm |= static_cast<unsigned>(act[j]) << j;
    unsigned over = mover;
    #pragma unroll 1
    while (over) {
      const int i = __builtin_ctz(over);
      over &= over - 1;
      unsigned bits = actm;
      #pragma unroll 1
      while (__any(bits != 0)) {
        const bool has = bits != 0;
        const int js = has ? __builtin_ctz(bits) : 0;
        bits &= bits - 1;
        walk(has, i, js);
      }
    }
    SUB_ADD(PH_SENS_GEOMS, t_geoms);
    return;
  }
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (m.rf_mode == 1) {
      if (act[j]) m.rf_static[k0 + j * stride] = dist[j];  // producer pass: the static hits
    } else if (act[j] && MRS_SD_OK(sd)) {
#ifdef MRS_DIAG_SD_SINK
      asm volatile("" ::"v"(dist[j]));  // diagnostic build: the ray result is kept live, not stored
#else
      sd[adr[j]] = dist[j];
#endif
    }
  }
  SUB_ADD(PH_SENS_GEOMS, t_geoms);
}

// the rangefinder passes of a model with more than 32 ray geoms: geoms in chunks of 32 (one mask bit
// each), every geom of a chunk a candidate (the level-1 blocks and the static split are built only
// for <= 32 ray geoms), each chunk continuing from the nearest hit so far in the ray's output slot
template <int G>
__device__ void rays_chunked(ENV_PARAMS, gfloat* sensordata) {
  ENV_UNPACK;
  constexpr int R = RayBatch<G>::value;
  const float zero[3] = {0, 0, 0};
  #pragma unroll 1
  for (int base = 0; base < m.nrf; base += G * R) {
    #pragma unroll 1
    for (int goff = 0; goff < m.nrgeom; goff += 32) {
      const int nc = m.nrgeom - goff;
      rangefinders<G, R, true>(m, s, sensordata, base + lane, G, nc >= 32 ? 0xffffffffu : ((1u << nc) - 1u), -1,
                               zero, goff);
    }
  }
}

// mj_sensorPos/Vel for the implemented sensor types; rangefinders lane-parallel within the group,
// RayBatch<G> rays per lane per pass
template <int G>
__device__ __forceinline__ void rays_pass(ENV_PARAMS, gfloat* sensordata) {
  ENV_UNPACK;
  if constexpr (G == 64) sensordata = uniform_ptr(sensordata);
  if (m.disableflags & MRS_DSBL_SENSOR) return;
  // level 1: which ray geoms can a ray block reach at all (fan bound of the block vs bounding sphere
  // of the geom; planes by the direction range of the fan), one bitmask per block; lanes over geoms
  const unsigned all = m.nrgeom >= 32 ? 0xffffffffu : ((1u << m.nrgeom) - 1u);
  unsigned long long t_l1 = SUB_T();
#if (defined(MRS_DIAG_RAYS) && MRS_DIAG_RAYS == 2) || defined(MRS_DIAG_NO_L1)
  if (false)  // diagnostic build: no level-1 test (all geoms)
#endif
  #pragma unroll 1
  for (int blk = 0; blk < m.nrfblk; ++blk) {
    const lfloat* br = shared_lds(m) + m.shr_blk + 16 * blk;  // staged from rfblk at launch
    unsigned mask = all;
    if (__float_as_int(br[1])) {
      const int b = __float_as_int(br[0]);
      const float ol[3] = {br[2], br[3], br[4]}, al[3] = {br[5], br[6], br[7]};
      const float bl[3] = {br[8], br[9], br[10]}, cl[3] = {br[11], br[12], br[13]};
      const float cth = br[14], sth = br[15], eps = shared_lds(m)[m.shr_blk + 16 * m.nrfblk + blk];
      float o[3], a[3], bb[3], c[3];
      if (m.rf_static_frame) {  // frame already in the world (static lidar)
        for (int i = 0; i < 3; ++i) { o[i] = ol[i]; a[i] = al[i]; bb[i] = bl[i]; c[i] = cl[i]; }
      } else {
        const float bq[4] = {s[L.xquat + 4 * b], s[L.xquat + 4 * b + 1], s[L.xquat + 4 * b + 2], s[L.xquat + 4 * b + 3]};
        float bmat[9];
        quat2mat(bmat, bq);
        mat_vec(o, bmat, ol);
        for (int i = 0; i < 3; ++i) o[i] += s[L.xpos + 3 * b + i];
        mat_vec(a, bmat, al);
        mat_vec(bb, bmat, bl);
        mat_vec(c, bmat, cl);
      }
      mask = 0;
      #pragma unroll 1
      for (int c0 = 0; c0 < m.nrgeom; c0 += G) {
        const int i = c0 + lane;
        bool cand = false;
        if (i < m.nrgeom) {
          const lfloat* rec = shared_lds(m) + 8 * i;
          const int g = __float_as_int(rec[0]), type = __float_as_int(rec[1]);
          const float v[3] = {s[L.gxpos + 3 * g] - o[0], s[L.gxpos + 3 * g + 1] - o[1], s[L.gxpos + 3 * g + 2] - o[2]};
          if (type == MRS_GEOM_PLANE) {
            // hit needs the origin in front of the plane and some ray direction with d.n < -1e-6
            // (the ray-plane test's parallel tolerance): d.n >= -(|(a.n, b.n)| + eps |c.n|)
            const float n[3] = {s[L.gxmat + 9 * g + 2], s[L.gxmat + 9 * g + 5], s[L.gxmat + 9 * g + 8]};
            const float An = dot3(a, n), Bn = dot3(bb, n), Cn = dot3(c, n);
            cand = -dot3(v, n) > 0 && sqrtf(An * An + Bn * Bn) + eps * fabsf(Cn) > 1e-6f;
          } else {
            const float rb = rec[3] * 1.0001f + 1e-6f;
            const float l2 = dot3(v, v);
            if (l2 <= rb * rb) {
              cand = true;
            } else {
              const float lv = sqrtf(l2);
              const float rr = rb + eps * (lv + rb);  // sphere radius plus out-of-plane drift
              const float wa = dot3(v, a), wb = dot3(v, bb), h = dot3(v, c);
              const float wn2 = wa * wa + wb * wb;
              // in-plane: angle(w, a) <= theta + asin(rb/|w|)  <=>  cos of it >= cos(theta + asin(rb/|w|)),
              // i.e. wa >= cos(theta) sqrt(|w|^2 - rb^2) - sin(theta) rb (theta + asin <= pi here);
              // rb is inflated by 0.1% + 1e-4 for rounding
              const float rbi = rb * 1.001f + 1e-4f;
              cand = fabsf(h) <= rr &&
                     (wn2 <= rbi * rbi || wa >= cth * sqrtf(wn2 - rbi * rbi) - sth * rbi);
            }
          }
        }
        const unsigned long long bal = __ballot(cand);
        const unsigned bits = static_cast<unsigned>((bal >> (__lane_id() & ~(G - 1))) & ((G == 64) ? ~0ull : ((1ull << G) - 1)));
        mask |= c0 < 32 ? bits << c0 : 0u;
      }
    }
    if (lane == 0) s[L.rfmask + blk] = __int_as_float(static_cast<int>(mask));
  }
  wsync();
  SUB_ADD(PH_SENS_L1, t_l1);
  // passes of G x R rays; lidars of more than one R = RayBatch pass take twice the rays per lane
  // (measured C3, 360 rays: 0.527 ms per launch at R = 8 vs 0.537 at 4, 0.560 at 10)
  auto passes = [&](auto rc) {
    constexpr int R = decltype(rc)::value;
    #pragma unroll 1
    for (int base = 0; base < m.nrf; base += G * R) {
      unsigned gmask = all;
  #if defined(MRS_DIAG_RAYS) && MRS_DIAG_RAYS == 2
      if (false) {
  #else
      if (m.nrfblk > 0) {
  #endif
        gmask = 0;
        const int b1 = min(m.nrfblk, (base + G * R + kRayBlock - 1) / kRayBlock);
        for (int blk = base / kRayBlock; blk < b1; ++blk) gmask |= static_cast<unsigned>(__float_as_int(s[L.rfmask + blk]));
      }
      // static split: the producer tests the world-welded geoms, the step the moving ones
      if (m.rf_mode == 1) gmask &= m.rf_static_mask;
      else if (m.rf_mode == 2) gmask &= ~m.rf_static_mask;
      // no geom reachable from this pass in any group of the wave: every ray misses (-1)
      unsigned wm = gmask;
      if constexpr (G < 64) {
  #pragma unroll
        for (int i = 0; i < 64 / G; ++i) wm |= __builtin_amdgcn_readlane(gmask, i * G);
      }
      if (__builtin_amdgcn_readfirstlane(wm) == 0) {
        // (static split: the static hit is the answer)
  #pragma unroll
        for (int j = 0; j < R; ++j) {
          const int k = base + lane + j * G;
          if (k >= m.nrf) continue;
          if (m.rf_mode == 1) m.rf_static[k] = -1.0f;
          else if (MRS_SD_OK(sensordata)) {
            const int adr = m.rf_common ? __float_as_int(shared_lds(m)[m.shr_rf + 4 * k + 3]) : __float_as_int(m.rfray[8 * k + 3]);
            sensordata[adr] = m.rf_mode == 2 ? (float)shared_lds(m)[m.shr_rfst + k] : -1.0f;
          }
        }
        continue;
      }
      // shared body and origin for the whole pass when all its blocks are fans from one point
      int common_body = -1;
      float common_o[3] = {0, 0, 0};
      const lfloat* blks = shared_lds(m) + m.shr_blk;
      if (m.rf_common) {
        common_body = __float_as_int(blks[0]);
        common_o[0] = blks[2]; common_o[1] = blks[3]; common_o[2] = blks[4];
      } else if (m.nrfblk > 0) {
        const int b0 = base / kRayBlock, b1 = min(m.nrfblk, (base + G * R + kRayBlock - 1) / kRayBlock);
        const lfloat* r0 = blks + 16 * b0;
        bool same = __float_as_int(r0[1]) != 0;
        for (int blk = b0 + 1; blk < b1 && same; ++blk) {
          const lfloat* ri = blks + 16 * blk;
          same = __float_as_int(ri[1]) != 0 && __float_as_int(ri[0]) == __float_as_int(r0[0]) && ri[2] == r0[2] &&
                 ri[3] == r0[3] && ri[4] == r0[4];
        }
        if (same) {
          common_body = __float_as_int(r0[0]);
          common_o[0] = r0[2]; common_o[1] = r0[3]; common_o[2] = r0[4];
        }
      }
      rangefinders<G, R>(m, s, sensordata, base + lane, G, gmask, common_body, common_o);
    }
  };
  if (m.nrgeom > 32) {
    // more ray geoms than mask bits: the chunked pass (rays_chunked) is called by the step loop
    // right after forward() returns, in the extended kernels (MRS_EXT)
  } else
#ifdef MRS_RAY_BATCH
  passes(std::integral_constant<int, MRS_RAY_BATCH>{});
#else
  // (a lidar of at most 2 G rays takes 2 per lane: one pass with no idle ray slots; C4's 32 beams)
  if (G < 64 && m.nrf > G * RayBatch<G>::value) passes(std::integral_constant<int, 2 * RayBatch<G>::value>{});
  else if (G < 64 && RayBatch<G>::value > 2 && m.nrf <= 2 * G) passes(std::integral_constant<int, 2>{});
  else passes(std::integral_constant<int, RayBatch<G>::value>{});
#endif
}

// the step's sensors: the rangefinder passes (rays: 0 when the workgroup's ray helper waves take them,
// step_kernel) and the other sensor types
template <int G>
__device__ MRS_PHASE void sensors(ENV_PARAMS, gfloat* sensordata, bool rays = true) {
  ENV_UNPACK;
  if constexpr (G == 64) sensordata = uniform_ptr(sensordata);
  if (m.disableflags & MRS_DSBL_SENSOR) return;
  if (rays) rays_pass<G>(ENV_ARGS, sensordata);
  if (!MRS_SD_OK(sensordata)) return;
#ifdef MRS_DIAG_NO_OTHER
  return;  // diagnostic build: rangefinders only
#endif
  #pragma unroll 1
  for (int ks = lane; ks < m.nsens_other; ks += G) {
    // the sensor's descriptor from workgroup LDS (batch.hip sensrec): no chain of dependent model loads
    const lfloat* sr = shared_lds(m) + m.shr_sens + 16 * ks;
    const int t = __float_as_int(sr[0]), id = __float_as_int(sr[14]), a = __float_as_int(sr[5]);
    gfloat* out = sensordata + __float_as_int(sr[2]);
    float cutoff = sr[4];
    int dim = __float_as_int(sr[3]);
    switch (t) {
      case MRS_SENS_RANGEFINDER: continue;
      case MRS_SENS_JOINTPOS: out[0] = s[L.qpos + a]; break;
      case MRS_SENS_JOINTVEL: out[0] = s[L.qvel + a]; break;
      case MRS_SENS_ACTUATORFRC: out[0] = s[L.act_force + id]; break;
      case MRS_SENS_ACCELEROMETER:
      case MRS_SENS_FORCE:
      case MRS_SENS_TORQUE: {
        // mj_sensorAcc: com-based quantities moved to the site (mju_transformSpatial), site frame
        const int b = a, rt = __float_as_int(sr[6]);
        float bq[4] = {s[L.xquat + 4 * b], s[L.xquat + 4 * b + 1], s[L.xquat + 4 * b + 2], s[L.xquat + 4 * b + 3]};
        float sp[3] = {sr[7], sr[8], sr[9]};
        float sq[4] = {sr[10], sr[11], sr[12], sr[13]};
        float r[3], q[4], sm[9], d[3], o3[3];
        rot_quat(r, sp, bq);
        for (int i = 0; i < 3; ++i) d[i] = s[L.xpos + 3 * b + i] + r[i] - s[L.scom + 3 * rt + i];
        quat_mul(q, bq, sq);
        quat2mat(sm, q);
        if (t == MRS_SENS_ACCELEROMETER) {
          // a_lin - d x a_ang + w x (v_lin - d x w), then into the site frame
          float w3[3], v3[3], a3[3], dw[3], da[3], acc[3];
          for (int i = 0; i < 3; ++i) {
            w3[i] = s[L.cvel + 6 * b + i];
            v3[i] = s[L.cvel + 6 * b + 3 + i];
            a3[i] = s[L.cacc + 6 * b + i];
          }
          cross3(dw, d, w3);
          cross3(da, d, a3);
          for (int i = 0; i < 3; ++i) v3[i] -= dw[i];
          cross3(acc, w3, v3);
          for (int i = 0; i < 3; ++i) acc[i] += s[L.cacc + 6 * b + 3 + i] - da[i];
          matT_vec(o3, sm, acc);
        } else {
          float tq[3], f3[3], df[3];
          for (int i = 0; i < 3; ++i) { tq[i] = s[L.crb + 6 * b + i]; f3[i] = s[L.crb + 6 * b + 3 + i]; }
          if (t == MRS_SENS_FORCE) {
            matT_vec(o3, sm, f3);
          } else {
            cross3(df, d, f3);
            for (int i = 0; i < 3; ++i) tq[i] -= df[i];
            matT_vec(o3, sm, tq);
          }
        }
        for (int i = 0; i < 3; ++i) out[i] = o3[i];
        break;
      }
      case MRS_SENS_FRAMEPOS:
      case MRS_SENS_FRAMEQUAT:
      case MRS_SENS_GYRO: {
        const int ot = __float_as_int(sr[1]);
        float p[3], q[4];
        int b;
        if (ot == MRS_OBJ_SITE || t == MRS_SENS_GYRO) {
          b = a;
          float bq[4] = {s[L.xquat + 4 * b], s[L.xquat + 4 * b + 1], s[L.xquat + 4 * b + 2], s[L.xquat + 4 * b + 3]};
          float sp[3] = {sr[7], sr[8], sr[9]};
          float sq[4] = {sr[10], sr[11], sr[12], sr[13]};
          float r[3];
          rot_quat(r, sp, bq);
          for (int i = 0; i < 3; ++i) p[i] = s[L.xpos + 3 * b + i] + r[i];
          quat_mul(q, bq, sq);
        } else if (ot == MRS_OBJ_BODY) {
          b = id;
          for (int i = 0; i < 3; ++i) p[i] = s[L.xpos + 3 * b + i];
          for (int i = 0; i < 4; ++i) q[i] = s[L.xquat + 4 * b + i];
        } else {
          b = a;
          float bq[4] = {s[L.xquat + 4 * b], s[L.xquat + 4 * b + 1], s[L.xquat + 4 * b + 2], s[L.xquat + 4 * b + 3]};
          float gq[4] = {sr[10], sr[11], sr[12], sr[13]};
          for (int i = 0; i < 3; ++i) p[i] = s[L.gxpos + 3 * id + i];
          quat_mul(q, bq, gq);
        }
        if (t == MRS_SENS_FRAMEPOS) { for (int i = 0; i < 3; ++i) out[i] = p[i]; }
        else if (t == MRS_SENS_FRAMEQUAT) { quat_normalize(q); for (int i = 0; i < 4; ++i) out[i] = q[i]; cutoff = 0; }
        else {
          float sm[9], w[3] = {s[L.cvel + 6 * b], s[L.cvel + 6 * b + 1], s[L.cvel + 6 * b + 2]};
          quat2mat(sm, q);
          float o3[3];
          matT_vec(o3, sm, w);
          for (int i = 0; i < 3; ++i) out[i] = o3[i];
        }
        break;
      }
      default:
        for (int i = 0; i < dim; ++i) out[i] = 0;
    }
    if (cutoff > 0)
      for (int i = 0; i < dim; ++i) out[i] = clampf(out[i], -cutoff, cutoff);
  }
}

// reset one env (mj_resetData; held inputs ctrl/qfrc_applied are re-applied by the caller's loop)
template <int G>
__device__ MRS_PHASE void reset_env(ENV_PARAMS) {
  ENV_UNPACK;
  #pragma unroll 1
  for (int i = lane; i < m.nq; i += G) s[L.qpos + i] = m.qpos0[i];
  #pragma unroll 1
  for (int i = lane; i < m.nv; i += G) { s[L.qvel + i] = 0; s[L.qacc_ws + i] = 0; }
  wsync();
}

template <int G>
__device__ MRS_PHASE bool any_bad(ENV_PARAMS, int off, int n) {
  ENV_UNPACK;
  off = uniform_int(off);
  n = uniform_int(n);
  bool bad = false;
  #pragma unroll 1
  for (int i = lane; i < n; i += G) bad |= is_bad(s[off + i]);
  return gany<G>(bad);
}

// mj_checkPos / mj_checkVel of the step loop: a vector of at most G entries is one LDS read per lane and
// a group vote, inline; longer ones take any_bad.  (The step loop keeps these checks off out-of-line
// calls: a call starts with the ABI's s_waitcnt vmcnt(0), which at the step boundary waited for the
// step's sensordata stores to land -- inlining the loop of any_bad instead cost C3 3 % in spills.)
template <int G>
__device__ __forceinline__ bool any_bad_step(ENV_PARAMS, int off, int n) {
  if (n <= G) return gany<G>(lane < n && is_bad(s[off + lane]));
  return any_bad<G>(ENV_ARGS, off, n);
}

template <int G>
__device__ __forceinline__ void cholesky_ih(ENV_PARAMS);

// full forward pass; returns the contact count.  With acc_bad, *acc_bad is the group's vote on qacc
// (mj_checkAcc), taken from the solver's lane-per-dof result in registers
template <int G, bool kPrimal = false, bool kHot = false>
__device__ MRS_PHASE int forward(ENV_PARAMS, gfloat* sensordata PH_ACC_PARAM, bool helper = false,
                                 bool* acc_bad = nullptr) {
  ENV_UNPACK;
  if constexpr (G == 64) sensordata = uniform_ptr(sensordata);
  PH_BEGIN();
  MRS_CALL(G, kinematics<G>(ENV_ARGS));
  // helper waves (step_kernel): the poses are in LDS -- release the helpers (barrier A); they run this
  // step's collision pass and trace its rays while the wave goes on, and nothing below writes what
  // they read
  if (helper) helper_barrier(false);
  PH_END(ph_acc, PH_KIN);
  MRS_CALL(G, com_pos<G>(ENV_ARGS));
  // helper waves: com_pos's cdof and subtree coms are in LDS -- signal the helper, which builds the
  // constraint rows from them after its collision pass (no wait here)
  if (helper && helper_rows(m)) helper_signal(m, __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6);
  PH_END(ph_acc, PH_COMPOS);
  MRS_CALL(G, make_M<G>(ENV_ARGS));
  PH_END(ph_acc, PH_MAKEM);
  if (G == 16 && m.fuse_ih) MRS_CALL(G, cholesky_ih<G>(ENV_ARGS));
  else MRS_CALL(G, cholesky<G>(mp, s + L.M, s + L.L, lane));
  PH_END(ph_acc, PH_CHOL);
  MRS_CALL(G, com_vel<G>(ENV_ARGS));
  PH_END(ph_acc, PH_COMVEL);
  MRS_CALL(G, rne<G>(ENV_ARGS));
  PH_END(ph_acc, PH_RNE);
  float qacc_s;
  MRS_CALL(G, qacc_s = smooth_forces<G>(ENV_ARGS));
  PH_END(ph_acc, PH_SMOOTH);
  int ncon = 0, pre_nefc = -1;
  if (helper) {
    // barrier C: the helper's contact records (and with helper_rows its constraint rows) are stored
    // -- its collision pass and rows ran beside the smooth dynamics above, which need neither
    helper_barrier(false);
    const int hc = __float_as_int(s[L.hcon]);
    ncon = hc & 0xffff;
    pre_nefc = (hc >> 16) - 1;
  } else if (!(m.diag_skip & 2)) {
    MRS_CALL(G, ncon = collision<G>(ENV_ARGS));
  }
  PH_END(ph_acc, PH_COLL);
  float qacc = qacc_s;
  if (lane == 0) {
    s[L.niter] = __int_as_float(0);
    // no rows unless constraints() builds some (mrs_batch_get_efc), or the helper's
    scr[S.efc_n] = __int_as_float(pre_nefc >= 0 ? pre_nefc : 0);
  }
  if (!(m.diag_skip & 4)) MRS_CALL(G, qacc = (constraints<G, kPrimal, kHot>(ENV_ARGS, ncon, qacc_s, pre_nefc)));
  PH_END(ph_acc, PH_CONSTR);
  if (lane < m.nv) s[L.qacc + lane] = qacc;
  if (acc_bad) *acc_bad = gany<G>(lane < m.nv && is_bad(qacc));
  wsync();
  // sensordata == nullptr: mj_forwardSkip(skipsensor) (the RK4 stages)
  if (sensordata) {
    if (m.acc_sens && !(m.disableflags & MRS_DSBL_SENSOR)) { [[clang::noinline]] rne_post<G>(ENV_ARGS, ncon); }
    if (!(m.diag_skip & 1)) MRS_CALL(G, sensors<G>(ENV_ARGS, sensordata, !helper));
  }
  PH_END(ph_acc, PH_SENS);
  return ncon;
}

// mj_integratePos: qpos (LDS) advanced by h * vel (an LDS vector of nv)
template <int G>
__device__ __forceinline__ void integrate_pos(const DevModel& m, lfloat* s, const lfloat* vel, float h, int lane) {
  const LdsLayout& L = m.L;
  #pragma unroll 1
  for (int j = lane; j < m.njnt; j += G) {
    const auto kj = kin_jnt<G>(m, j);  // (workgroup LDS with lane groups: no global load right after
    //                                   the step's sensordata stores, which it would wait for)
    int a = __float_as_int(kj[6]), da = __float_as_int(kj[10]);
    const int jt = __float_as_int(kj[7]);
    if (jt == MRS_JNT_HINGE || jt == MRS_JNT_SLIDE) {
      s[L.qpos + a] += h * vel[da];
      continue;
    }
    if (jt == MRS_JNT_FREE) {
      for (int i = 0; i < 3; ++i) s[L.qpos + a + i] += h * vel[da + i];
      a += 3; da += 3;
    }
    float q[4] = {s[L.qpos + a], s[L.qpos + a + 1], s[L.qpos + a + 2], s[L.qpos + a + 3]};
    float v[3] = {vel[da], vel[da + 1], vel[da + 2]};
    float ang = h * normalize3(v), dq[4];
    axis_angle_quat(dq, v, ang);
    quat_normalize(q);
    quat_mul(q, q, dq);
    quat_normalize(q);
    for (int i = 0; i < 4; ++i) s[L.qpos + a + i] = q[i];
  }
  wsync();
}

template <int G>
__device__ void integrate_implicit(ENV_PARAMS);

// the integrator's implicit damping of lane's dof (mj_Euler: dof damping; implicitfast: damping and
// the actuators' velocity derivatives), 0 past nv
template <int G>
__device__ __forceinline__ float integrate_dg(ENV_PARAMS) {
  ENV_UNPACK;
  const int nv = m.nv;
  float dg = 0;
  if (lane < nv) {
    const auto dr = dof_tab<G>(m, lane);
    const float damping = dr[9];
    if (m.integrator == MRS_INT_EULER) {
      if (!(m.disableflags & MRS_DSBL_EULERDAMP) && damping > 0) dg = damping;
    } else {
      if (!(m.disableflags & MRS_DSBL_PASSIVE)) dg = damping;
      if (!(m.disableflags & MRS_DSBL_ACTUATION)) {
        // velocity derivative of the actuators on this dof (the dof's single actuator from its
        // table row; several: every actuator is checked)
        auto act_dv = [&](int a) {
          const auto ar = act_tab<G>(m, a);
          if (__float_as_int(ar[14])) {
            const float f = s[L.act_force + a];
            if (f <= ar[15] || f >= ar[16]) return;
          }
          const float bv = __float_as_int(ar[10]) == MRS_BIAS_AFFINE ? ar[13] : 0.0f;
          const float gv = __float_as_int(ar[6]) == MRS_GAIN_AFFINE ? ar[9] : 0.0f;
          float ctrl = s[L.ctrl + a];
          if (__float_as_int(ar[3]) && !(m.disableflags & MRS_DSBL_CLAMPCTRL)) ctrl = clampf(ctrl, ar[4], ar[5]);
          const float g = ar[2];
          dg -= g * g * (bv + gv * ctrl);
        };
        const int da = __float_as_int(dr[0]);
        if (da >= 0) {
          act_dv(da);
        } else if (da == -2) {
          #pragma unroll 1
          for (int a = 0; a < m.nu; ++a)
            if (__float_as_int(act_tab<G>(m, a)[1]) == lane) act_dv(a);
        }
      }
    }
  }
  return dg;
}

// the helper waves' share of the integrator (step_kernel): M + h diag(dg) factored into L.Lh while
// the physics wave runs the constraint solve (M, the dof damping, ctrl and the actuator forces of the
// step are final by then); integrate() then only solves.  Returns nothing when no solve is needed.
template <int G>
__device__ __forceinline__ void integrate_prefactor(ENV_PARAMS) {
  ENV_UNPACK;
  const int nv = m.nv;
  const float dg = integrate_dg<G>(ENV_ARGS);
  if (!(m.integrator != MRS_INT_EULER || gany<G>(dg != 0))) return;
  const float h = m.timestep;
  #pragma unroll 1
  for (int j = 0; j < nv; ++j)
    if (lane < nv) s[L.Lh + midx<G>(m, lane, j)] = s[L.M + midx<G>(m, lane, j)];
  // (the diagonal update in the same statement form as integrate()'s in-place M_ii += h dg, so it
  // contracts the same way: one fma, bit-identical factors)
  if (lane < nv) s[L.Lh + midx<G>(m, lane, lane)] += h * dg;
  wsync();
  MRS_CALL(G, cholesky<G>(mp, s + L.Lh, s + L.Lh, lane));
}

// M's factor (L.L) and, for integrate(), the factor of M + h D (DevModel::fuse_ih: 16-lane implicitfast
// models) in M's slot for PGS, whose M is not read after the factor, in L.Lh for Newton / CG
template <int G>
__device__ __forceinline__ void cholesky_ih(ENV_PARAMS) {
  ENV_UNPACK;
  if constexpr (G == 16) {
    const float dg = integrate_dg<G>(ENV_ARGS);
    lfloat* ih = s + (m.solver == MRS_SOL_PGS ? L.M : L.Lh);
    if (m.nv <= 8) chol_rows16_dual<8>(s + L.M, s + L.L, ih, m.timestep, dg, m.nv, lane);
    else chol_rows16_dual<16>(s + L.M, s + L.L, ih, m.timestep, dg, m.nv, lane);
    wsync();
  }
}

// mj_Euler / mj_implicit(implicitfast) + mj_advance (prefac: the factor of M + h D is in L.Lh, built
// by the helper wave, or with DevModel::fuse_ih in L.M, built beside M's factor)
template <int G>
__device__ MRS_PHASE void integrate(ENV_PARAMS, bool prefac = false) {
  ENV_UNPACK;
  if (m.integrator == MRS_INT_IMPLICIT) {
    [[clang::noinline]] integrate_implicit<G>(ENV_ARGS);
    return;
  }
  const int nv = m.nv;
  const float h = m.timestep;
  const float qacc = lane < nv ? s[L.qacc + lane] : 0.0f;
  const float dg = integrate_dg<G>(ENV_ARGS);
  const bool need_solve = m.integrator != MRS_INT_EULER || gany<G>(dg != 0);
  float qacc_int = qacc;
  if (need_solve) {
    const float rhs = lane < nv ? s[L.qfrc_smooth + lane] + s[L.qfrc_con + lane] : 0.0f;
    if (prefac) {
      MRS_CALL(G, qacc_int = chol_solve_lanes<G>(mp, s + (m.fuse_ih && m.solver == MRS_SOL_PGS ? L.M : L.Lh), rhs, lane));
    } else {
      // M + h*diag(dg) into the M slot (M is rebuilt every step), factor into L
      if (lane < nv) s[L.M + midx<G>(m, lane, lane)] += h * dg;
      wsync();
      MRS_CALL(G, cholesky<G>(mp, s + L.M, s + L.L, lane));
      MRS_CALL(G, qacc_int = chol_solve_lanes<G>(mp, s + L.L, rhs, lane));
    }
  }
  if (lane < nv) {
    s[L.qacc_ws + lane] = qacc;
    s[L.qvel + lane] += h * qacc_int;
  }
  wsync();
  integrate_pos<G>(m, s, s + L.qvel, h, lane);
}

// the velocity derivative of the actuators and passive forces on lane j's dof, as integrate()'s
// implicitfast path (minus the derivative of qfrc_passive + qfrc_actuator)
template <int G>
__device__ __forceinline__ float implicit_dg(const DevModel& m, const lfloat* s, int lane) {
  const LdsLayout& L = m.L;
  const auto dr = dof_tab<G>(m, lane);
  float dg = (m.disableflags & MRS_DSBL_PASSIVE) ? 0.0f : dr[9];
  if (!(m.disableflags & MRS_DSBL_ACTUATION)) {
    auto act_dv = [&](int a) {
      const auto ar = act_tab<G>(m, a);
      if (__float_as_int(ar[14])) {
        const float f = s[L.act_force + a];
        if (f <= ar[15] || f >= ar[16]) return;
      }
      const float bv = __float_as_int(ar[10]) == MRS_BIAS_AFFINE ? ar[13] : 0.0f;
      const float gv = __float_as_int(ar[6]) == MRS_GAIN_AFFINE ? ar[9] : 0.0f;
      float ctrl = s[L.ctrl + a];
      if (__float_as_int(ar[3]) && !(m.disableflags & MRS_DSBL_CLAMPCTRL)) ctrl = clampf(ctrl, ar[4], ar[5]);
      const float g = ar[2];
      dg -= g * g * (bv + gv * ctrl);
    };
    const int da = __float_as_int(dr[0]);
    if (da >= 0) {
      act_dv(da);
    } else if (da == -2) {
      #pragma unroll 1
      for (int a = 0; a < m.nu; ++a)
        if (__float_as_int(act_tab<G>(m, a)[1]) == lane) act_dv(a);
    }
  }
  return dg;
}

// mj_implicit with the full velocity derivative (oracle.c integrate / orc_bias_vel): the matrix
// M + h (diag(dg) + d qfrc_bias / d qvel) is not symmetric (Coriolis, centrifugal and gyroscopic
// terms), so it is factored by LU without pivoting.  Column j of the RNE derivative is
// (bias(qvel + e_j) - bias(qvel - e_j)) / 2 -- exact for qfrc_bias, which is quadratic in qvel -- from
// two com_vel + rne passes of the env's own phases; the derivative couples only dofs of one kinematic
// tree, so blocked mode keeps M's tree blocks and factors each in place (lane = row of its tree).
// Out of line: only models with integrator="implicit" reach it.
// After it returns, qvel is restored but the velocity-dependent LDS fields of the last perturbed
// pass (cvel, cdofdot, cacc, cfrc / crb and qfrc_bias) hold the state at qvel - e_j: nothing reads
// them before the next step's forward() recomputes them; a post-integrate consumer would have to
// rerun com_vel + rne first.
template <int G>
__device__ void integrate_implicit(ENV_PARAMS) {
  ENV_UNPACK;
  const int nv = m.nv;
  const float h = m.timestep;
  const float qacc = lane < nv ? s[L.qacc + lane] : 0.0f;
  const float dg = lane < nv ? implicit_dg<G>(m, s, lane) : 0.0f;
  const float rhs = lane < nv ? s[L.qfrc_smooth + lane] + s[L.qfrc_con + lane] : 0.0f;
  int ta = 0, tn = nv, tmax = nv;
  if constexpr (G == 64) {
    tmax = m.tree_nmax;
    if (lane < nv) {
      const int t = m.dof_tree[lane];
      ta = m.tree_dofadr[t];
      tn = m.tree_dofnum[t];
    }
  }
  if (lane < nv) s[L.M + midx<G>(m, lane, lane)] += h * dg;
  #pragma unroll 1
  for (int j = 0; j < nv; ++j) {
    const float vj = s[L.qvel + j];
    float bias[2];
    for (int sg = 0; sg < 2; ++sg) {
      wsync();
      if (lane == 0) s[L.qvel + j] = sg == 0 ? vj + 1.0f : vj - 1.0f;
      wsync();
      com_vel<G>(ENV_ARGS);
      rne<G>(ENV_ARGS);
      bias[sg] = lane < nv ? s[L.qfrc_bias + lane] : 0.0f;
    }
    wsync();
    if (lane == 0) s[L.qvel + j] = vj;
    if (lane < nv && j >= ta && j < ta + tn) s[L.M + midx<G>(m, lane, j)] += h * (0.5f * (bias[0] - bias[1]));
  }
  // (the velocity-stage LDS fields -- cvel, cdofdot, cacc, cfrc / crb, qfrc_bias -- are left at the
  // last perturbed velocity; nothing reads them before the next step's forward() recomputes them)
  wsync();
  auto from = [&](float v, int src) {  // the value of lane src of this env's group
    if constexpr (G == 64) return __shfl(v, src);
    else return gbcast<G>(v, src);
  };
  // LU of every tree block in place (unit lower L below the diagonal, U on and above)
  #pragma unroll 1
  for (int k = 0; k < tmax; ++k) {
    const int piv = ta + k;
    if (lane < nv && k < tn && lane - ta > k) {
      const float l = s[L.M + midx<G>(m, lane, piv)] / s[L.M + midx<G>(m, piv, piv)];
      s[L.M + midx<G>(m, lane, piv)] = l;
      #pragma unroll 1
      for (int c = k + 1; c < tn; ++c) s[L.M + midx<G>(m, lane, ta + c)] -= l * s[L.M + midx<G>(m, piv, ta + c)];
    }
    wsync();
  }
  float y = rhs;
  #pragma unroll 1
  for (int k = 0; k < tmax; ++k) {
    const float yk = from(y, min(ta + k, G - 1));
    if (lane < nv && k < tn && lane - ta > k) y -= s[L.M + midx<G>(m, lane, ta + k)] * yk;
  }
  float x = 0;
  #pragma unroll 1
  for (int k = tmax - 1; k >= 0; --k) {
    if (lane < nv && lane - ta == k) x = y / s[L.M + midx<G>(m, lane, lane)];
    const float xk = from(x, min(ta + k, G - 1));
    if (lane < nv && k < tn && lane - ta < k) y -= s[L.M + midx<G>(m, lane, ta + k)] * xk;
  }
  if (lane < nv) {
    s[L.qacc_ws + lane] = qacc;
    s[L.qvel + lane] += h * x;
  }
  wsync();
  integrate_pos<G>(m, s, s + L.qvel, h, lane);
}

// mj_RungeKutta(m, d, 4) (oracle.c rk4 states the restatement): the stages around the step loop's
// single forward() call site.  Stage i = 1..3 (entered with F_{i-1} = (qvel, qacc) in LDS): saves X_0
// at stage 1, accumulates B_{i-1} F_{i-1}, and sets X_i = X_0 '+' h A_i F_{i-1}; rk4_final adds F_3
// and advances X_0 by h sum B_j F_j.  Lane per dof (nv <= G); qpos lane-strided.
template <int G>
__device__ void rk4_stage(ENV_PARAMS, int stage) {
  ENV_UNPACK;
  const int nq = m.nq, nv = m.nv;
  const float h = m.timestep;
  const float a = stage == 3 ? 1.0f : 0.5f;
  const float b = stage == 1 ? 1.0f / 6 : 1.0f / 3;
  lfloat* q0 = s + L.rk;
  lfloat* v0 = q0 + (nq > 1 ? nq : 1);
  lfloat *dv = v0 + nv, *sv = dv + nv, *sa = sv + nv;
  if (stage == 1) {
    #pragma unroll 1
    for (int i = lane; i < nq; i += G) q0[i] = s[L.qpos + i];
  }
  #pragma unroll 1
  for (int j = lane; j < nv; j += G) {
    const float vel = s[L.qvel + j], acc = s[L.qacc + j];
    if (stage == 1) {
      v0[j] = vel;
      sv[j] = b * vel;
      sa[j] = b * acc;
    } else {
      sv[j] += b * vel;
      sa[j] += b * acc;
    }
    dv[j] = a * vel;
    s[L.qvel + j] = v0[j] + h * (a * acc);
  }
  #pragma unroll 1
  for (int i = lane; i < nq; i += G) s[L.qpos + i] = q0[i];
  wsync();
  integrate_pos<G>(m, s, dv, h, lane);
}
template <int G>
__device__ void rk4_final(ENV_PARAMS) {
  ENV_UNPACK;
  const int nq = m.nq, nv = m.nv;
  const float h = m.timestep;
  lfloat* q0 = s + L.rk;
  lfloat* v0 = q0 + (nq > 1 ? nq : 1);
  lfloat *sv = v0 + 2 * nv, *sa = sv + nv;
  #pragma unroll 1
  for (int j = lane; j < nv; j += G) {
    const float acc = s[L.qacc + j];
    sv[j] += (1.0f / 6) * s[L.qvel + j];
    const float dA = sa[j] + (1.0f / 6) * acc;
    s[L.qacc_ws + j] = acc;  // mj_advance: the last stage's qacc
    s[L.qvel + j] = v0[j] + h * dA;
  }
  #pragma unroll 1
  for (int i = lane; i < nq; i += G) s[L.qpos + i] = q0[i];
  wsync();
  integrate_pos<G>(m, s, sv, h, lane);
}

// waves per SIMD the register budget is sized for.  One env per wave (G = 64, blocked mode): 2 waves
// (256 VGPRs) -- the register-resident sparse PGS holds up to 64 rows per pipe, and the per-env LDS of
// the multi-tree scenes that pick G = 64 (C5: ~13 KB) allows ~2 waves per SIMD anyway.  With G < 64
// the LDS of 4*64/G envs per workgroup bounds residency instead (e.g. G = 16: 16 envs x 4.5 KB per
// workgroup -> 2 workgroups per CU -> 2 waves per SIMD, 256 VGPRs)
template <int G>
#ifndef MRS_G64_WAVES
#define MRS_G64_WAVES 2
#endif
#ifndef MRS_G16_OCC
#define MRS_G16_OCC 2
#endif
struct Occupancy { static constexpr int waves = G == 64 ? MRS_G64_WAVES : (G == 32 ? 4 : (G == 16 ? MRS_G16_OCC : 1)); };

// kHelpers: the G = 16 step kernel with ray helper waves (DevState::ray_helpers; its own instantiation,
// so the kernels without helpers keep their code and registers -- the run-time switch alone cost C3 5%)
template <int G, bool kForwardOnly, bool kPrimal = false, bool kHelpers = false>
// the helper-wave kernels at one wave per SIMD (up to 512 VGPRs: the physics wave keeps its values in
// registers around the out-of-line dense constraint path instead of spilling them, and the frames
// rendered beside the steps overlap them better; C4 31.5 -> 32.5 M, under Newton 27.7 -> 28.1 M,
// same-box A/B): batch.hip takes helpers only while physics and helper waves together fit one per
// SIMD
#ifndef MRS_HELPER_OCC
#define MRS_HELPER_OCC 1
#endif
__global__ __launch_bounds__(64 * WavesPerBlock<G>::value, kHelpers ? MRS_HELPER_OCC : Occupancy<G>::waves) void step_kernel(
    const DevModel* __restrict__ mp, DevState st, int n_envs, int n_steps) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int kEnvsPerBlock = G == 16 ? 4 * st.wpb16 : WavesPerBlock<G>::value * 64 / G;
  const DevModel& m = *mp;
  const LdsLayout& L = m.L;
  // ray helper waves (DevState::ray_helpers, G = 16 step launches): the workgroup's second half, wave
  // w + wpb16 tracing the rangefinders of physics wave w's envs each step between two barriers
  constexpr bool helpers = G == 16 && !kForwardOnly && kHelpers;
  const bool is_helper = helpers && threadIdx.x >= 64 * st.wpb16;
  const int tid = is_helper ? threadIdx.x - 64 * st.wpb16 : threadIdx.x;
  const int lane = tid & (G - 1), slot = tid / G;
  // group -> env: with spread 2^k (DevState::spread_shift), 2^k consecutive groups step one env and
  // only the first writes back (the others mirror it: same state, same arithmetic, own scratch), so
  // a small batch occupies 2^k times the waves (C4's 2048 envs: 512 waves on 1024 SIMDs otherwise)
  const int vgroup = blockIdx.x * kEnvsPerBlock + slot;
  const int env = vgroup >> st.spread_shift;
  const bool primary = (vgroup & ((1 << st.spread_shift) - 1)) == 0;
  // groups past n_envs (and mirrors) stay alive (the wave-cooperative ray phase needs every lane) and
  // step a valid env with their own scratch; they write nothing back
  const bool valid = env < n_envs && primary;
  lfloat* s = (lfloat*)(smem + slot * L.total);
  gfloat* scr = (gfloat*)(st.scratch + (size_t)(valid || st.spread_shift == 0 ? env : st.scr_mirror + vgroup) * m.S.total);
  const size_t e = (size_t)(env < n_envs ? env : n_envs - 1);
  #pragma unroll 1
  for (int i = lane; i < (is_helper ? 0 : m.nq); i += G) s[L.qpos + i] = st.qpos[e * m.nq + i];
  #pragma unroll 1
  for (int i = lane; i < (is_helper ? 0 : m.nv); i += G) {
    s[L.qvel + i] = st.qvel[e * m.nv + i];
    s[L.qfrc_applied + i] = st.qfrc_applied[e * m.nv + i];
    s[L.qacc_ws + i] = st.qacc_ws[e * m.nv + i];
  }
  #pragma unroll 1
  for (int i = lane; i < (is_helper ? 0 : m.nu); i += G) s[L.ctrl + i] = st.ctrl[e * m.nu + i];
  if constexpr (G == 64) {
    #pragma unroll 1
    for (int t = lane; t < m.ntree; t += G) {
      s[L.trees + 4 * t] = __int_as_float(m.tree_dofadr[t]);
      s[L.trees + 4 * t + 1] = __int_as_float(m.tree_dofnum[t]);
      s[L.trees + 4 * t + 2] = __int_as_float(m.tree_Moff[t]);
      s[L.trees + 4 * t + 3] = 0;
    }
    #pragma unroll 1
    for (int j = lane; j < m.nv; j += G) {
      const int bj = m.dof_bodyid[j];
      s[L.dofb + 2 * j] = __int_as_float(bj);
      s[L.dofb + 2 * j + 1] = __int_as_float(m.body_subtree_end[bj]);
    }
  }
  double time = st.time[e];
  gfloat* sensordata = valid ? (gfloat*)(st.sensordata + e * m.nsensordata) : scr + m.S.sens;
  {
    // workgroup-shared tables (DevModel::shr_*): ray-geom records and per-ray direction + address
    float* shr = smem + m.shr_off;
    #pragma unroll 1
    for (int i = threadIdx.x; i < m.shr_rf; i += blockDim.x) shr[i] = m.rgeom[i];
    #pragma unroll 1
    for (int i = threadIdx.x; i < m.shr_rfst - m.shr_rf; i += blockDim.x) shr[m.shr_rf + i] = m.rfray[8 * (i >> 2) + (i & 3)];
    if (m.rf_mode == 2)
      #pragma unroll 1
      for (int i = threadIdx.x; i < m.nrf; i += blockDim.x) shr[m.shr_rfst + i] = m.rf_static[i];
    #pragma unroll 1
    for (int i = threadIdx.x; i < 17 * m.nrfblk; i += blockDim.x) shr[m.shr_blk + i] = m.rfblk[i];
    #pragma unroll 1
    for (int i = threadIdx.x; i < 16 * m.nsens_other; i += blockDim.x) shr[m.shr_sens + i] = m.sensrec[i];
    #pragma unroll 1
    for (int i = threadIdx.x; i < 4 * m.nfric; i += blockDim.x) shr[m.shr_fric + i] = m.fricrec[i];
    #pragma unroll 1
    for (int i = threadIdx.x; i < 4 * m.nlim; i += blockDim.x) shr[m.shr_lim + i] = m.limrec[i];
    if constexpr (G < 64) {  // smooth-dynamics tables (blocked mode reads the model block)
      #pragma unroll 1
      for (int i = threadIdx.x; i < 20 * m.nu; i += blockDim.x) shr[m.shr_act + i] = m.actrec[i];
      #pragma unroll 1
      for (int i = threadIdx.x; i < 16 * m.nv; i += blockDim.x) shr[m.shr_dof + i] = m.dofrec[i];
      #pragma unroll 1
      for (int i = threadIdx.x; i < 8 * m.nbody; i += blockDim.x) shr[m.shr_body + i] = m.bodytab[i];
      #pragma unroll 1
      for (int i = threadIdx.x; i < 4 * m.nMpair; i += blockDim.x) shr[m.shr_mpair + i] = m.mpairtab[i];
      #pragma unroll 1
      for (int i = threadIdx.x; i < m.njump * m.nbody; i += blockDim.x) shr[m.shr_jump + i] = __int_as_float(m.jump[i]);
      #pragma unroll 1
      for (int i = threadIdx.x; i < 25 * m.nbody; i += blockDim.x) shr[m.shr_kbody + i] = m.kinbody[i];
      #pragma unroll 1
      for (int i = threadIdx.x; i < 13 * m.njnt; i += blockDim.x) shr[m.shr_kjnt + i] = m.kinjnt[i];
      #pragma unroll 1
      for (int i = threadIdx.x; i < 9 * m.ngeom; i += blockDim.x) shr[m.shr_kgeom + i] = m.kingeom[i];
    }
  }
  if (helpers && threadIdx.x < 4) *helper_flag(m, threadIdx.x) = 0;
  __syncthreads();
  wsync();
  if (is_helper) {
    // barrier A (the physics wave's poses are in LDS), the collision pass, barrier C (contacts
    // stored, their count in LDS), the rays, barrier B (results stored); the physics waves pass A, C
    // and B exactly once per step (forward() after kinematics and before constraints, then below)
    // with helper_rows also the dense constraint rows, after the physics wave's signal that its
    // com_pos outputs are in LDS (helper_wait); their count goes to LDS with the contact count
    const int hwave = (__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6) - st.wpb16;  // its physics wave
    int timeouts = 0;
    #pragma unroll 1
    for (int step = 0; step < n_steps; ++step) {
      helper_barrier(false);
      int nc = 0, nr = -1;
      if (!(m.diag_skip & 2)) MRS_CALL(G, nc = collision<G>(ENV_ARGS));
      if (helper_rows(m)) {
        // the physics wave's com_pos of this step is done; on a timeout (a protocol fault) nr stays
        // -1 and the physics wave builds the rows itself
        if (helper_wait(m, hwave, step + 1)) {
          [[clang::noinline]] nr = dense_rows<G>(ENV_ARGS, nc);
          MRS_CALL(G, dense_impedance<G>(ENV_ARGS, nr));
        } else {
          ++timeouts;
        }
      }
      if (lane == 0) s[L.hcon] = __int_as_float(nc + 65536 * (nr + 1));
      helper_barrier(true);
      MRS_CALL(G, rays_pass<G>(ENV_ARGS, sensordata));
      // the integrator's factor of M + h D (the physics wave solves with it after B)
      if (L.Lh != 0) MRS_CALL(G, integrate_prefactor<G>(ENV_ARGS));
      helper_barrier(true);
    }
    if (timeouts && valid && lane == 0) st.warning[4 * e + 3] += timeouts;
    return;
  }
  int ncon = 0;
  int w_pos = 0, w_vel = 0, w_acc = 0;
#ifdef MRS_PHASE_TIMING
  unsigned long long ph_acc[PH_COUNT] = {};
#endif
  for (int step = 0; step < n_steps; ++step) {
    if (!kForwardOnly) {
      if (any_bad_step<G>(ENV_ARGS, L.qpos, m.nq)) {
        ++w_pos;
        if (!(m.disableflags & MRS_DSBL_AUTORESET)) { [[clang::noinline]] reset_env<G>(ENV_ARGS); time = 0; }
      }
      if (any_bad_step<G>(ENV_ARGS, L.qvel, m.nv)) {
        ++w_vel;
        if (!(m.disableflags & MRS_DSBL_AUTORESET)) { [[clang::noinline]] reset_env<G>(ENV_ARGS); time = 0; }
      }
    }
#ifdef MRS_DIAG_SENS_LAST
    // diagnostic build: sensors evaluated and stored on the last step of the launch only
    gfloat* sd_step = (kForwardOnly || step == n_steps - 1) ? sensordata : nullptr;
#else
    gfloat* sd_step = sensordata;
#endif
    bool acc_bad = false;
    MRS_CALL(G, ncon = (forward<G, kPrimal, helpers && !kPrimal>(ENV_ARGS, sd_step PH_ACC_ARG, helpers, &acc_bad)));
    if (helpers) helper_barrier(false);  // barrier B: this step's rays are stored
#if MRS_EXT
    // rangefinders of a model with more than 32 ray geoms (sensors() leaves them to this call)
    if (m.nrgeom > 32 && m.nrf > 0 && !(m.disableflags & MRS_DSBL_SENSOR))
      [[clang::noinline]] rays_chunked<G>(ENV_ARGS, sd_step);
#endif
    if (kForwardOnly) break;
    bool redo = false;
    if (acc_bad) {
      ++w_acc;
      if (!(m.disableflags & MRS_DSBL_AUTORESET)) {
        [[clang::noinline]] reset_env<G>(ENV_ARGS);
        time = 0;
        redo = true;
      }
    }
    // forward() is entered by the whole wave; for envs that were not reset it recomputes the
    // same outputs from the same state
    if (__any(redo)) {  // rare
      [[clang::noinline]] ncon = forward<G, kPrimal>(ENV_ARGS, sd_step PH_ACC_ARG);
#if MRS_EXT
      if (m.nrgeom > 32 && m.nrf > 0 && !(m.disableflags & MRS_DSBL_SENSOR))
        [[clang::noinline]] rays_chunked<G>(ENV_ARGS, sd_step);
#endif
    }
    if (m.integrator == MRS_INT_RK4) {
      // stages out of line (RK4 models only), each followed by a forward without sensors
      #pragma unroll 1
      for (int stage = 1; stage < 4; ++stage) {
        [[clang::noinline]] rk4_stage<G>(ENV_ARGS, stage);
        [[clang::noinline]] ncon = forward<G, kPrimal>(ENV_ARGS, nullptr PH_ACC_ARG);
      }
      [[clang::noinline]] rk4_final<G>(ENV_ARGS);
    } else {
      PH_BEGIN();
      // (a re-run step's factor is its own: the helper's was of the first forward's state)
      MRS_CALL(G, integrate<G>(ENV_ARGS, (helpers && L.Lh != 0 && !__any(redo)) || (G == 16 && m.fuse_ih)));
      PH_END(ph_acc, PH_INTEG);
    }
    time += m.timestep_d;
  }
#ifdef MRS_PHASE_TIMING
  if (__lane_id() == 0)
    for (int i = 0; i < PH_COUNT; ++i) atomicAdd(&g_phase_cycles[i], ph_acc[i]);
#endif
  if (!valid) return;
  // kinematics of the last forward pass (what mjv_updateScene would render after mj_step)
  #pragma unroll 1
  for (int i = lane; i < 3 * m.ngeom; i += G) st.geom_xpos[e * 3 * m.ngeom + i] = s[L.gxpos + i];
  #pragma unroll 1
  for (int i = lane; i < 9 * m.ngeom; i += G) st.geom_xmat[e * 9 * m.ngeom + i] = s[L.gxmat + i];
  #pragma unroll 1
  for (int c = lane; c < m.ncam; c += G) {
    const int b = m.cam_bodyid[c];
    float bq[4] = {s[L.xquat + 4 * b], s[L.xquat + 4 * b + 1], s[L.xquat + 4 * b + 2], s[L.xquat + 4 * b + 3]};
    float cp[3] = {m.cam_pos[3 * c], m.cam_pos[3 * c + 1], m.cam_pos[3 * c + 2]};
    float cq[4] = {m.cam_quat[4 * c], m.cam_quat[4 * c + 1], m.cam_quat[4 * c + 2], m.cam_quat[4 * c + 3]};
    float r[3], q[4], cm[9];
    rot_quat(r, cp, bq);
    quat_mul(q, bq, cq);
    quat2mat(cm, q);
    for (int i = 0; i < 3; ++i) st.cam_xpos[(e * m.ncam + c) * 3 + i] = s[L.xpos + 3 * b + i] + r[i];
    for (int i = 0; i < 9; ++i) st.cam_xmat[(e * m.ncam + c) * 9 + i] = cm[i];
  }
  #pragma unroll 1
  for (int i = lane; i < m.nq; i += G) st.qpos[e * m.nq + i] = s[L.qpos + i];
  #pragma unroll 1
  for (int i = lane; i < m.nv; i += G) {
    st.qvel[e * m.nv + i] = s[L.qvel + i];
    st.qacc_ws[e * m.nv + i] = s[L.qacc_ws + i];
    st.qacc[e * m.nv + i] = s[L.qacc + i];
    st.qfrc_act[e * m.nv + i] = s[L.qfrc_act + i];
  }
  if (lane == 0) {
    st.time[e] = time;
    st.ncon[e] = ncon;
    st.niter[e] = __float_as_int(s[L.niter]);
    if (w_pos | w_vel | w_acc) {  // (warning[3] is the helper wave's: its signal timeouts)
      st.warning[4 * e + 0] += w_pos;
      st.warning[4 * e + 1] += w_vel;
      st.warning[4 * e + 2] += w_acc;
    }
  }
}

}  // namespace

// kernel selection bits of launch_g (the split build compiles each part in its own translation unit)
constexpr int kSelForward = 1, kSelStep = 2, kSelPrimal = 4, kSelHelpers = 8, kSelAll = 15;

template <int G, int kSel = kSelAll>
static void launch_g(const DevModel* d_model, int lds_floats, int shared_floats, const DevState& st, int n_envs,
                     int n_steps, bool forward_only, bool primal, hipStream_t stream) {
  const int wpb = G == 16 ? st.wpb16 : WavesPerBlock<G>::value;
  const int kEnvsPerBlock = wpb * 64 / G;
  const int blocks = ((n_envs << st.spread_shift) + kEnvsPerBlock - 1) / kEnvsPerBlock;
  const size_t lds = sizeof(float) * ((size_t)lds_floats * kEnvsPerBlock + shared_floats);
  if constexpr (G == 16 && (kSel & kSelHelpers)) {
    // step launches with ray helper waves: twice the waves per workgroup
    if (st.ray_helpers && !forward_only) {
      if (primal)
        hipLaunchKernelGGL((step_kernel<G, false, true, true>), dim3(blocks), dim3(128 * wpb), lds, stream, d_model, st,
                           n_envs, n_steps);
      else
        hipLaunchKernelGGL((step_kernel<G, false, false, true>), dim3(blocks), dim3(128 * wpb), lds, stream, d_model, st,
                           n_envs, n_steps);
      return;
    }
  }
  if constexpr (G == 16 && (kSel & kSelPrimal)) {
    if (primal && !forward_only) {
      hipLaunchKernelGGL((step_kernel<G, false, true>), dim3(blocks), dim3(64 * wpb), lds, stream, d_model, st,
                         n_envs, n_steps);
      return;
    }
  }
  if constexpr ((kSel & kSelForward) != 0) {
    if (forward_only) {
      hipLaunchKernelGGL((step_kernel<G, true>), dim3(blocks), dim3(64 * wpb), lds, stream, d_model, st, n_envs, 1);
      return;
    }
  }
  if constexpr ((kSel & kSelStep) != 0) {
    if (!forward_only)
      hipLaunchKernelGGL((step_kernel<G, false>), dim3(blocks), dim3(64 * wpb), lds, stream, d_model, st, n_envs,
                         n_steps);
  }
}

#if !defined(MRS_STEP_PART) || MRS_STEP_PART == 0
// profiling variant only: per-phase wave-cycle totals since the last reset (s_memtime ticks summed
// over waves); returns the number of phases, 0 in normal builds
int phase_cycles(double* out, int n, bool reset) {
#ifdef MRS_PHASE_TIMING
  unsigned long long h[PH_COUNT];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase_cycles), sizeof h) != hipSuccess) return -1;
  for (int i = 0; i < PH_COUNT && i < n; ++i) out[i] = static_cast<double>(h[i]);
  if (reset) {
    unsigned long long z[PH_COUNT] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof z) != hipSuccess) return -1;
  }
  return PH_COUNT;
#else
  (void)out; (void)n; (void)reset;
  return 0;
#endif
}

#endif

#ifndef MRS_STEP_PART
// single translation unit: every instantiation (the variant builds, scripts/build_variant.sh)
hipError_t launch_step(const DevModel* d_model, int lds_floats, int shared_floats, const DevState& st, int n_envs,
                       int n_steps, bool forward_only, int group, bool primal, bool ext, hipStream_t stream) {
  (void)ext;  // (one translation unit: MRS_EXT as compiled)
  switch (group) {
    case 8: launch_g<8>(d_model, lds_floats, shared_floats, st, n_envs, n_steps, forward_only, primal, stream); break;
    case 16: launch_g<16>(d_model, lds_floats, shared_floats, st, n_envs, n_steps, forward_only, primal, stream); break;
    case 32: launch_g<32>(d_model, lds_floats, shared_floats, st, n_envs, n_steps, forward_only, primal, stream); break;
    case 64: launch_g<64>(d_model, lds_floats, shared_floats, st, n_envs, n_steps, forward_only, primal, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
#else
// split build (build.py): step.hip is compiled once per part, in parallel, each part instantiating
// only its own kernels; part 0 holds the dispatcher.  Parts 16 / 17 (G = 16 primal) / 64 are compiled
// without the extended code (MRS_EXT 0: the MPR contact polish and the chunked pass of more than 32
// ray geoms -- their call sites alone cost the inlined G = 16 / 64 phases registers and scratch: C3
// -1.3% for the ray call site); models that need it run parts 18 (G = 16) / 65 (G = 64), and the
// G = 8 / 32 parts always carry it
#define MRS_LAUNCH_ARGS const DevModel* d_model, int lds_floats, int shared_floats, const DevState& st, int n_envs, \
                        int n_steps, bool forward_only, bool primal, hipStream_t stream
#define MRS_LAUNCH_PASS d_model, lds_floats, shared_floats, st, n_envs, n_steps, forward_only, primal, stream
void launch_part_8(MRS_LAUNCH_ARGS);
void launch_part_16(MRS_LAUNCH_ARGS);
void launch_part_17(MRS_LAUNCH_ARGS);
void launch_part_18(MRS_LAUNCH_ARGS);
void launch_part_19(MRS_LAUNCH_ARGS);
void launch_part_32(MRS_LAUNCH_ARGS);
void launch_part_64(MRS_LAUNCH_ARGS);
void launch_part_65(MRS_LAUNCH_ARGS);
#if MRS_STEP_PART == 0
hipError_t launch_step(const DevModel* d_model, int lds_floats, int shared_floats, const DevState& st, int n_envs,
                       int n_steps, bool forward_only, int group, bool primal, bool ext, hipStream_t stream) {
  switch (group) {
    case 8: launch_part_8(MRS_LAUNCH_PASS); break;
    case 16:
      if (ext) launch_part_18(MRS_LAUNCH_PASS);
      else if (st.ray_helpers && !forward_only) launch_part_19(MRS_LAUNCH_PASS);
      else if (primal && !forward_only) launch_part_17(MRS_LAUNCH_PASS);
      else launch_part_16(MRS_LAUNCH_PASS);
      break;
    case 32: launch_part_32(MRS_LAUNCH_PASS); break;
    case 64:
      if (ext) launch_part_65(MRS_LAUNCH_PASS);
      else launch_part_64(MRS_LAUNCH_PASS);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
#elif MRS_STEP_PART == 16
void launch_part_16(MRS_LAUNCH_ARGS) { launch_g<16, kSelForward | kSelStep>(MRS_LAUNCH_PASS); }
#elif MRS_STEP_PART == 17
void launch_part_17(MRS_LAUNCH_ARGS) { launch_g<16, kSelPrimal>(MRS_LAUNCH_PASS); }
#elif MRS_STEP_PART == 18
void launch_part_18(MRS_LAUNCH_ARGS) { launch_g<16, kSelForward | kSelStep | kSelPrimal>(MRS_LAUNCH_PASS); }
#elif MRS_STEP_PART == 19
// G = 16 step kernels (PGS and primal) with ray helper waves, without the extended code
void launch_part_19(MRS_LAUNCH_ARGS) { launch_g<16, kSelHelpers>(MRS_LAUNCH_PASS); }
#elif MRS_STEP_PART == 65
void launch_part_65(MRS_LAUNCH_ARGS) { launch_g<64>(MRS_LAUNCH_PASS); }
#else
#define MRS_PART_FN2(n) launch_part_##n
#define MRS_PART_FN(n) MRS_PART_FN2(n)
void MRS_PART_FN(MRS_STEP_PART)(MRS_LAUNCH_ARGS) { launch_g<MRS_STEP_PART>(MRS_LAUNCH_PASS); }
#endif
#endif

}  // namespace mrs
