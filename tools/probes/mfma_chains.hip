// Probe: f64 MFMA throughput against dependency-chain length and waves per SIMD.  Each wave issues
// NCH independent accumulation chains of v_mfma_f64_16x16x4, round robin, ITER * 8 MFMAs in all; with
// NCH = 1 every MFMA waits for the previous one's result (the staged Gram kernel's transform and Gram
// chains are 4-5 long).  Occupancy is set by dynamic LDS per workgroup (4 waves each): 1, 2 or 4 waves
// per SIMD.  Prints TF/s against the 78.6 TF/s dense fp64 peak.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NCH>
__global__ __launch_bounds__(256) void k_chain(double* out, int iters, double s) {
  extern __shared__ double pad[];
  d4 acc[NCH];
#pragma unroll
  for (int q = 0; q < NCH; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  const double a = s * threadIdx.x, b = s * 2.0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) acc[m % NCH] = __builtin_amdgcn_mfma_f64_16x16x4f64(a + m, b, acc[m % NCH], 0, 0, 0);
  }
  double t = 0.0;
#pragma unroll
  for (int q = 0; q < NCH; ++q) t += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  if (t == 12345.0) pad[threadIdx.x] = t;     // never: keeps the LDS allocation
  out[size_t(blockIdx.x) * 256 + threadIdx.x] = t;
}

template <int NCH>
void run(double* out, int ncu, int wps) {
  // LDS per 4-wave workgroup so that wps workgroups fit a CU (160 KB): wps waves per SIMD
  const size_t lds = size_t(160 * 1024 / wps) - 1024;
  const int blocks = ncu * wps * 8, iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_chain<NCH>, dim3(blocks), dim3(256), lds, 0, out, 10, 1e-9);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_chain<NCH>, dim3(blocks), dim3(256), lds, 0, out, iters, 1e-9);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = double(blocks) * 4 * iters * 8 * 2048.0;
  printf("{\"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"TFs\": %.1f}\n", NCH, wps, ms, flops / ms / 1e9);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  double* out;
  hipMalloc(&out, size_t(p.multiProcessorCount) * 4 * 8 * 256 * sizeof(double));
  for (int wps : {1, 2, 4}) {
    run<1>(out, p.multiProcessorCount, wps);
    run<2>(out, p.multiProcessorCount, wps);
    run<4>(out, p.multiProcessorCount, wps);
  }
  return 0;
}
