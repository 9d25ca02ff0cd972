// Colour of a camera pixel: the lit model oracle.c lit_color / sky_color / tex_sample restate in fp64
// (MuJoCo's fixed-function OpenGL render -- mjr_render, reached from src/mujoco_cameras.cpp:211-240 --
// evaluated per pixel): per light (the headlight first, then the model's active lights)
//   c += att spot (amb base + sh (max(0, N.L) dif base + [N.L > 0] max(0, N.H)^(128 shin) spc specular))
// on top of emission * base, N the normal facing the viewer, E the view axis, H = normalize(L + E),
// sh = 0 when the ray from the surface towards a castshadow light hits a geom first.  Everything is
// evaluated in the camera frame: the frame's lights are staged once per workgroup (lit_stage) with
// their positions and directions rotated into it, so a pixel needs only its ray slope, hit distance
// and camera-frame normal.  rlit (DevModel::rlit, packed by build_devmodel) holds, in floats:
//   [0, 12)              headlight ambient[3] diffuse[3] specular[3] active, nlight, sky texture id
//   12 + 24 l            light l: pos[3] dir[3] ambient[3] diffuse[3] specular[3] attenuation[3]
//                        cos(cutoff) exponent directional castshadow active (pad)
//   mat0 + 12 m          material m: texid texuniform texrepeat[2] specular shininess emission
//   tex0 + 16 t          texture t: type builtin mark width height rgb1[3] rgb2[3] markrgb[3]
#pragma once

constexpr int kLitHead = 12, kLitLight = 24, kLitMat = 12, kLitTex = 16, kLitMaxLights = 8;

struct LitRef {
  const float* rlit;
  const int* geom_matid;  // -1: no material
  int nlight, mat0, tex0, sky;  // sky: first skybox texture, -1 none
};

struct LitLight {
  float L[3];    // directional: unit vector towards the light; else the light position (camera frame)
  float dir[3];  // spot axis (camera frame)
  float amb[3], dif[3], spc[3], att[3];
  float cosc, expo;
  int directional, shadow;
};
struct LitFrame {
  int n;
  int sky;           // -1 none, 1 gradient, 0 two-colour (flat / checker)
  float c1[3], c2[3];
  float up[3];       // world z in the camera frame: the sky's dz of a ray d is up.d / |d|
  LitLight l[kLitMaxLights + 1];
};

// one thread of the workgroup fills the frame's light table (camera pose: cpos, rotation C with the
// camera axes as columns); the caller synchronises before the pixels read it
__device__ inline void lit_stage(LitFrame& F, const LitRef& lr, const float cpos[3], const float C[9]) {
  const float* r = lr.rlit;
  int n = 0;
  if (r[9] != 0) {
    LitLight& h = F.l[n++];
    for (int i = 0; i < 3; ++i) {
      h.L[i] = i == 2 ? 1.0f : 0.0f;
      h.dir[i] = 0;
      h.amb[i] = r[i]; h.dif[i] = r[3 + i]; h.spc[i] = r[6 + i];
      h.att[i] = 0;
    }
    h.cosc = -2; h.expo = 0; h.directional = 1; h.shadow = 0;
  }
  for (int l = 0; l < lr.nlight; ++l) {
    const float* s = r + kLitHead + kLitLight * l;
    if (s[22] == 0) continue;
    LitLight& o = F.l[n++];
    const float d[3] = {s[0] - cpos[0], s[1] - cpos[1], s[2] - cpos[2]};
    for (int i = 0; i < 3; ++i) {
      const float dc = C[i] * s[3] + C[3 + i] * s[4] + C[6 + i] * s[5];  // C' dir
      o.dir[i] = dc;
      o.L[i] = s[20] != 0 ? -dc : C[i] * d[0] + C[3 + i] * d[1] + C[6 + i] * d[2];
      o.amb[i] = s[6 + i]; o.dif[i] = s[9 + i]; o.spc[i] = s[12 + i]; o.att[i] = s[15 + i];
    }
    if (s[20] != 0) {
      const float nn = rsqrtf(fmaxf(o.L[0] * o.L[0] + o.L[1] * o.L[1] + o.L[2] * o.L[2], 1e-30f));
      for (int i = 0; i < 3; ++i) o.L[i] *= nn;
    }
    o.cosc = s[18]; o.expo = s[19]; o.directional = s[20] != 0; o.shadow = s[21] != 0;
  }
  F.n = n;
  F.sky = -1;
  for (int i = 0; i < 3; ++i) { F.c1[i] = F.c2[i] = 0; F.up[i] = C[6 + i]; }
  if (lr.sky >= 0) {
    const float* t = r + lr.tex0 + kLitTex * lr.sky;
    F.sky = t[1] == MRS_BUILTIN_GRADIENT ? 1 : 0;
    for (int i = 0; i < 3; ++i) { F.c1[i] = t[5 + i]; F.c2[i] = t[8 + i]; }
  }
}

__device__ __forceinline__ void lit_store(const float c[3], unsigned char* px) {
  for (int i = 0; i < 3; ++i) px[i] = static_cast<unsigned char>(fminf(fmaxf(c[i], 0.0f), 1.0f) * 255.0f + 0.5f);
}

// a pixel whose ray (dx, dy, -1) hits nothing: the skybox (oracle.c sky_color), else black
__device__ __forceinline__ void lit_sky(const LitFrame& F, float dx, float dy, unsigned char* px) {
  float c[3] = {0, 0, 0};
  if (F.sky >= 0) {
    const float dz = (F.up[0] * dx + F.up[1] * dy - F.up[2]) * rsqrtf(dx * dx + dy * dy + 1.0f);
    for (int i = 0; i < 3; ++i)
      c[i] = F.sky == 1 ? F.c2[i] + (F.c1[i] - F.c2[i]) * 0.5f * (1 + dz) : (dz >= 0 ? F.c1[i] : F.c2[i]);
  }
  lit_store(c, px);
}

// nearest texel of builtin texture t at (u, v) (oracle.c tex_sample)
__device__ __forceinline__ void lit_texel(const float* tx, float u, float v, float out[3]) {
  const int W = static_cast<int>(tx[3]), H = static_cast<int>(tx[4]);
  u -= floorf(u);
  v -= floorf(v);
  const int iu = min(max(static_cast<int>(u * W), 0), W - 1), iv = min(max(static_cast<int>(v * H), 0), H - 1);
  const int builtin = static_cast<int>(tx[1]), mark = static_cast<int>(tx[2]);
  const float *c1 = tx + 5, *c2 = tx + 8;
  if (builtin == MRS_BUILTIN_CHECKER) {
    const float* c = ((iu < W / 2) == (iv < H / 2)) ? c1 : c2;
    for (int i = 0; i < 3; ++i) out[i] = c[i];
  } else if (builtin == MRS_BUILTIN_GRADIENT) {
    const float s = H > 1 ? static_cast<float>(iv) / (H - 1) : 0.0f;
    for (int i = 0; i < 3; ++i) out[i] = c1[i] + s * (c2[i] - c1[i]);
  } else {
    for (int i = 0; i < 3; ++i) out[i] = c1[i];
  }
  if ((mark == MRS_MARK_EDGE && (iu == 0 || iv == 0 || iu == W - 1 || iv == H - 1)) ||
      (mark == MRS_MARK_CROSS && (iu == W / 2 || iv == H / 2)))
    for (int i = 0; i < 3; ++i) out[i] = tx[11 + i];
}

// the lit colour of a hit: geom g (colour rgba, type, size), geom-frame hit point q (plane texture
// coordinates), ray slope (dx, dy), hit distance t along (dx, dy, -1), camera-frame normal nc (any
// length, either orientation).  occluded(o, L, dist): a shadow-casting geom is hit by the ray o + s L,
// 0 <= s < dist (camera frame, L unit).
template <class Occ>
__device__ inline void lit_pixel(const LitFrame& F, const LitRef& lr, int g, const float rgba[3], int type,
                                 const float* size, const float q[3], float dx, float dy, float t,
                                 const float nc[3], Occ&& occluded, unsigned char* px) {
  const float v[3] = {dx, dy, -1.0f};
  float N[3] = {nc[0], nc[1], nc[2]};
  {
    const float nn = rsqrtf(fmaxf(N[0] * N[0] + N[1] * N[1] + N[2] * N[2], 1e-30f));
    const float s = (N[0] * v[0] + N[1] * v[1] + N[2] * v[2]) > 0 ? -nn : nn;
    for (int i = 0; i < 3; ++i) N[i] *= s;
  }
  float base[3] = {rgba[0], rgba[1], rgba[2]}, spec_m = 0.5f, shin = 0.5f, emis = 0.0f;
  const int mat = lr.geom_matid ? lr.geom_matid[g] : -1;
  if (mat >= 0) {
    const float* mr = lr.rlit + lr.mat0 + kLitMat * mat;
    spec_m = mr[4]; shin = mr[5]; emis = mr[6];
    const int tid = static_cast<int>(mr[0]);
    if (tid >= 0 && type == MRS_GEOM_PLANE) {
      const float* tx = lr.rlit + lr.tex0 + kLitTex * tid;
      if (tx[0] == MRS_TEX_2D) {
        float sc[2];
        for (int k = 0; k < 2; ++k) sc[k] = mr[2 + k] * (mr[1] != 0 || size[k] <= 0 ? 1.0f : 1.0f / (2 * size[k]));
        float tc[3];
        lit_texel(tx, q[0] * sc[0], q[1] * sc[1], tc);
        for (int i = 0; i < 3; ++i) base[i] *= tc[i];
      }
    }
  }
  const float P[3] = {t * dx, t * dy, -t};
  float c[3] = {emis * base[0], emis * base[1], emis * base[2]};
  for (int l = 0; l < F.n; ++l) {
    const LitLight& s = F.l[l];
    float L[3] = {s.L[0], s.L[1], s.L[2]}, att = 1, spot = 1, dist = 3.0e38f;
    if (!s.directional) {
      for (int i = 0; i < 3; ++i) L[i] -= P[i];
      dist = sqrtf(L[0] * L[0] + L[1] * L[1] + L[2] * L[2]);
      const float inv = dist > 0 ? 1.0f / dist : 0.0f;
      for (int i = 0; i < 3; ++i) L[i] *= inv;
      att = 1.0f / (s.att[0] + s.att[1] * dist + s.att[2] * dist * dist);
      const float ca = -(L[0] * s.dir[0] + L[1] * s.dir[1] + L[2] * s.dir[2]);
      spot = ca < s.cosc ? 0.0f : powf(ca, s.expo);
    }
    const float nl = fmaxf(0.0f, N[0] * L[0] + N[1] * L[1] + N[2] * L[2]);
    float sh = 1;
    if (s.shadow && nl > 0) {
      const float o[3] = {P[0] + 1e-4f * N[0], P[1] + 1e-4f * N[1], P[2] + 1e-4f * N[2]};
      if (occluded(o, L, dist)) sh = 0;
    }
    float Hv[3] = {L[0], L[1], L[2] + 1.0f};
    const float hn = rsqrtf(fmaxf(Hv[0] * Hv[0] + Hv[1] * Hv[1] + Hv[2] * Hv[2], 1e-30f));
    const float nh = fmaxf(0.0f, (N[0] * Hv[0] + N[1] * Hv[1] + N[2] * Hv[2]) * hn);
    const float sp = nl > 0 ? powf(nh, 128.0f * shin) : 0.0f;
    const float k = att * spot;
    for (int i = 0; i < 3; ++i) c[i] += k * (s.amb[i] * base[i] + sh * (nl * s.dif[i] * base[i] + sp * s.spc[i] * spec_m));
  }
  lit_store(c, px);
}
