// Probe (diagnostic, GPU): cycles per row of the 16-lane register PGS sweep's dependent chain
// (step.hip pgs_small16: med3 of the owner's residual -> s_nop 1 + v_fmac_f32_dpp row_newbcast into
// every lane's residual), one wave alone on the device, timed with s_memtime over 12-row sweeps; and
// the same chain without the DPP broadcast (plain v_fmac) and the broadcast through a separate
// v_mov_dpp, for comparison.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int K>
__device__ __forceinline__ float fmac_rowb(float acc, float a, float v) {
  asm("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : "+v"(acc) : "v"(v), "v"(a), "n"(K));
  return acc;
}
template <int K>
__device__ __forceinline__ float rowb(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150 + K, 0xf, 0xf, true));
}
template <int MODE>
__global__ void chain(float* out, unsigned long long* cyc, int sweeps) {
  const int lane = threadIdx.x & 15;
  float gn = 0.001f * lane, lo = -1.0f, hi = 1.0f, a[12];
  for (int r = 0; r < 12; ++r) a[r] = -0.01f * (r + lane + 1);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < sweeps; ++it) {
#define ROW(r)                                                              \
  {                                                                         \
    const float c = __builtin_amdgcn_fmed3f(gn, lo, hi);                    \
    if (MODE == 0) gn = fmac_rowb<r>(gn, a[r], c);                          \
    else if (MODE == 1) gn = __builtin_fmaf(a[r], c, gn);                   \
    else gn = __builtin_fmaf(a[r], rowb<r>(c), gn);                         \
  }
    ROW(0) ROW(1) ROW(2) ROW(3) ROW(4) ROW(5) ROW(6) ROW(7) ROW(8) ROW(9) ROW(10) ROW(11)
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = gn;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  float* d;
  unsigned long long* c;
  hipMalloc(&d, 64 * sizeof(float));
  hipMalloc(&c, sizeof(unsigned long long));
  const int sweeps = 10000;
  const char* name[3] = {"med3 -> s_nop 1 + v_fmac_f32_dpp row_newbcast", "med3 -> v_fmac (no broadcast)",
                         "med3 -> v_mov_dpp -> v_fma"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      if (mode == 0) hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, d, c, sweeps);
      if (mode == 1) hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, d, c, sweeps);
      if (mode == 2) hipLaunchKernelGGL(chain<2>, dim3(1), dim3(64), 0, 0, d, c, sweeps);
      hipDeviceSynchronize();
    }
    unsigned long long h;
    hipMemcpy(&h, c, sizeof h, hipMemcpyDeviceToHost);
    printf("%-48s %.1f s_memtime ticks per row\n", name[mode], double(h) / (12.0 * sweeps));
  }
  return 0;
}
