// Probe (diagnostic, GPU): checks the operand / result layout the blocked-mode Newton Hessian assumes
// for v_mfma_f32_16x16x4f32 on gfx950: lane l supplies A[l % 16][l / 16] and B[l / 16][l % 16] and
// receives D[4 (l / 16) + v][l % 16] in result register v.  Prints the max |D - A B| over random data.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void probe(const float* A, const float* B, float* D) {
  const int l = threadIdx.x, i = l & 15, k = l >> 4;
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(A[i * 4 + k], B[k * 16 + i], c, 0, 0, 0);
  for (int v = 0; v < 4; ++v) D[(4 * k + v) * 16 + i] = c[v];
}
int main() {
  float hA[64], hB[64], hD[256];
  for (int i = 0; i < 64; ++i) { hA[i] = rand() / (float)RAND_MAX - 0.5f; hB[i] = rand() / (float)RAND_MAX - 0.5f; }
  float *dA, *dB, *dD;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dD, sizeof hD);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double ref = 0;
      for (int k = 0; k < 4; ++k) ref += (double)hA[i * 4 + k] * hB[k * 16 + j];
      err = fmax(err, fabs(ref - hD[i * 16 + j]));
    }
  printf("mfma_f32_16x16x4f32 layout check: max |D - AB| = %g -> %s\n", err, err < 1e-5 ? "OK" : "MISMATCH");
  return err < 1e-5 ? 0 : 1;
}
