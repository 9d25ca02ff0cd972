// Probe (diagnostic, GPU): operand / result lane layout of v_mfma_f32_16x16x1f32 (4 blocks of 16x16x1)
// on gfx950.  Run 1: A = lane + 1, B = 1 -> D = the A lane + 1 feeding each result; run 2: A = 1,
// B = lane + 1 -> the B lane.  Prints, per result register r and lane l, "r l a_lane b_lane".
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v16f __attribute__((ext_vector_type(16)));
__global__ void probe(float* out, int mode) {
  const int l = threadIdx.x;
  const float a = mode == 0 ? float(l + 1) : 1.0f;
  const float b = mode == 0 ? 1.0f : float(l + 1);
  v16f c = {};
  v16f d = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) out[r * 64 + l] = d[r];
}
int main() {
  float *d, h[2][1024];
  hipMalloc(&d, 1024 * sizeof(float));
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h[mode], d, sizeof h[mode], hipMemcpyDeviceToHost);
  }
  for (int r = 0; r < 16; ++r)
    for (int l = 0; l < 64; ++l) printf("%d %d %d %d\n", r, l, int(h[0][r * 64 + l]) - 1, int(h[1][r * 64 + l]) - 1);
  hipFree(d);
  return 0;
}
