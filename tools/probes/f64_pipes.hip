// Probe: do f64 MFMA and f64 VALU FMA overlap on one SIMD?  Three kernels with the same
// per-wave work: MFMA only, VALU FMA only, both interleaved (independent chains throughout).
// Build: hipcc --offload-arch=gfx950 -O3 -o f64_pipes f64_pipes.hip ; run: ./f64_pipes
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, int iters, double s) {
  d4 acc[4] = {};
  double v[16];
  for (int j = 0; j < 16; ++j) v[j] = s * (threadIdx.x + j);
  const double a = s * threadIdx.x, b = s * 2.0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (MODE & 1) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b + q, acc[q], 0, 0, 0);
      if (MODE & 2) {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = fma(v[j], b, a);   // 16 FMAs ~ one MFMA's 1024 MACs / 64 lanes
      }
    }
  }
  double t = 0;
  for (int q = 0; q < 4; ++q) t += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  for (int j = 0; j < 16; ++j) t += v[j];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}
int main() {
  double* out;
  hipMalloc(&out, 256 * 4096 * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 2000;
  for (int rep = 0; rep < 2; ++rep) {
    float ms[4];
    for (int mode = 1; mode <= 3; ++mode) {
      hipEventRecord(e0);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-9);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-9);
      if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-9);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms[mode], e0, e1);
    }
    const double waves = blocks * 4.0, mf = waves * iters * 4, fm = waves * iters * 4 * 16 * 64;
    printf("mfma-only %.3f ms (%.1f TF/s)  valu-only %.3f ms (%.1f TF/s)  both %.3f ms (sum %.3f, max %.3f)\n",
           ms[1], mf * 2048 / ms[1] / 1e9, ms[2], fm * 2 / ms[2] / 1e9, ms[3], ms[1] + ms[2],
           ms[1] > ms[2] ? ms[1] : ms[2]);
  }
  return 0;
}
