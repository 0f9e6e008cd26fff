// Probe: v_mfma_f64_4x4x4_4b_f64 on gfx950 -- operand layout and throughput against the 16x16x4 form.
// Layout: experiment e puts a one-hot 1 in lane e of A and 1000 + lane in B; every non-zero output lane
// o then holds B of the lane that pairs with A's lane e, so {o: B lane} reads off the (block, i, k, j) maps.
// Throughput: NCH independent chains, 8 MFMAs per iteration, 2 waves per SIMD; TF/s against 78.6.
// hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(double* out) {
  const int e = blockIdx.x, l = threadIdx.x;
  const double a = l == e ? 1.0 : 0.0, b = 1000.0 + l;
  out[e * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}

template <int NCH, bool SMALL>
__global__ __launch_bounds__(256) void k_chain(double* out, int iters, double s) {
  const double a = s * threadIdx.x, b = s * 2.0;
  double t = 0.0;
  if constexpr (SMALL) {
    double acc[NCH];
#pragma unroll
    for (int q = 0; q < NCH; ++q) acc[q] = 0.0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < 8; ++m) acc[m % NCH] = __builtin_amdgcn_mfma_f64_4x4x4f64(a + m, b, acc[m % NCH], 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NCH; ++q) t += acc[q];
  } else {
    d4 acc[NCH];
#pragma unroll
    for (int q = 0; q < NCH; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < 8; ++m) acc[m % NCH] = __builtin_amdgcn_mfma_f64_16x16x4f64(a + m, b, acc[m % NCH], 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NCH; ++q) t += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  }
  out[size_t(blockIdx.x) * 256 + threadIdx.x] = t;
}

template <int NCH, bool SMALL>
void run(double* out, int ncu) {
  const int blocks = ncu * 2, iters = 4000;   // 4-wave workgroups, 2 per CU: 2 waves per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k_chain<NCH, SMALL>), dim3(blocks), dim3(256), 0, 0, out, 10, 1e-9);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_chain<NCH, SMALL>), dim3(blocks), dim3(256), 0, 0, out, iters, 1e-9);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double per = SMALL ? 512.0 : 2048.0;
  const double flops = double(blocks) * 4 * iters * 8 * per;
  const double cyc = ms * 1e-3 * 2.4e9 / (double(blocks) * 4 * iters * 8 / (ncu * 4));
  printf("{\"mfma\": \"%s\", \"chains\": %d, \"ms\": %.3f, \"TFs\": %.2f, \"cycles_per_mfma_per_simd_at_2.4GHz\": %.1f}\n",
         SMALL ? "f64_4x4x4_4b" : "f64_16x16x4", NCH, ms, flops / ms / 1e9, cyc);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  double* out;
  hipMalloc(&out, size_t(p.multiProcessorCount) * 2 * 256 * sizeof(double) + 64 * 64 * sizeof(double));
  hipLaunchKernelGGL(k_layout, dim3(64), dim3(64), 0, 0, out);
  double h[64 * 64];
  hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  for (int e = 0; e < 64; ++e) {
    printf("{\"a_lane\": %d, \"out\": {", e);
    bool first = true;
    for (int o = 0; o < 64; ++o)
      if (h[e * 64 + o] != 0.0) {
        printf("%s\"%d\": %d", first ? "" : ", ", o, int(h[e * 64 + o] - 1000.0));
        first = false;
      }
    printf("}}\n");
  }
  run<1, true>(out, p.multiProcessorCount);
  run<4, true>(out, p.multiProcessorCount);
  run<8, true>(out, p.multiProcessorCount);
  run<1, false>(out, p.multiProcessorCount);
  run<4, false>(out, p.multiProcessorCount);
  return 0;
}
