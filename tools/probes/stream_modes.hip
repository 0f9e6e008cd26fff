// Read-stream probe for the first-trial kernel's access pattern: x = sum_j c_j V_j over
// K columns of an N x N slab, one grid row at a time, written back with non-temporal stores.
//   mode 0: k_gemv_vjpg's current form -- a row-strided grid of the resident workgroups, each lane loads
//           its 2 points of all K columns of a row into VGPRs (nt loads), then computes;
//   mode 1: the same with the next row's loads issued before this row's compute (register prefetch);
//   mode 2: per-wave LDS-DMA ring (global_load_lds_dwordx4, default policy): every wave streams its own
//           128 points of R rows ahead into LDS and reads them back; no workgroup barriers;
//   mode 3: mode 2 with non-temporal DMA (aux = 2).
// Prints GB/s (K reads + 1 write per point) per mode and K.  hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) const void* glb_cvp;

#define CHK(x)                                                                       \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int BLOCK = 256;

template <int K, bool PF>
__global__ __launch_bounds__(BLOCK) void k_vgpr(const double* __restrict__ V, int64_t ldv, const double* __restrict__ cv,
                                                double* __restrict__ x, int64_t N) {
  const int64_t iy = (int64_t(blockIdx.x) * BLOCK + threadIdx.x) * 2;
  double c[K];
#pragma unroll
  for (int j = 0; j < K; ++j) c[j] = cv[j];
  if (iy >= N) return;
  d2 vv[K], vn[K];
  int64_t row = blockIdx.y;
  if (PF && row < N) {
#pragma unroll
    for (int j = 0; j < K; ++j) vn[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(V + j * ldv + row * N + iy));
  }
  for (; row < N; row += gridDim.y) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (PF) vv[j] = vn[j];
      else vv[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(V + j * ldv + row * N + iy));
    }
    if (PF && row + gridDim.y < N) {
#pragma unroll
      for (int j = 0; j < K; ++j)
        vn[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(V + j * ldv + (row + gridDim.y) * N + iy));
    }
    d2 s = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < K; ++j) {
      s.x = s.x + vv[j].x * c[j];
      s.y = s.y + vv[j].y * c[j];
    }
    __builtin_nontemporal_store(s, reinterpret_cast<d2*>(x + row * N + iy));
  }
}

constexpr unsigned waitcnt_vm(int n) { return unsigned((n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8)); }

// per-wave ring: R slots x K columns x 128 points (1 KB per column-row)
template <int K, int R, int AUX>
__global__ __launch_bounds__(BLOCK) void k_dma(const double* __restrict__ V, int64_t ldv, const double* __restrict__ cv,
                                               double* __restrict__ x, int64_t N) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double* ring = lds + size_t(wave) * R * K * 128;
  const int64_t iy = (int64_t(blockIdx.x) * BLOCK + threadIdx.x) * 2;    // 4 waves x 128 points
  const int64_t col0 = (int64_t(blockIdx.x) * BLOCK + wave * 64) * 2;
  double c[K];
#pragma unroll
  for (int j = 0; j < K; ++j) c[j] = cv[j];
  const int64_t row0 = blockIdx.y, rs = gridDim.y;
  auto issue = [&](int64_t row, int slot) {
    const int64_t rr = row < N ? row : N - 1;                 // past the end: re-load the last row
#pragma unroll
    for (int j = 0; j < K; ++j)
      __builtin_amdgcn_global_load_lds((glb_cvp)(V + j * ldv + rr * N + col0 + 2 * lane),
                                       (lds_vp)(ring + (slot * K + j) * 128), 16, 0, AUX);
  };
#pragma unroll
  for (int s = 0; s < R - 1; ++s) issue(row0 + s * rs, s);
  int slot = 0;
  for (int64_t row = row0; row < N; row += rs) {
    issue(row + (R - 1) * rs, (slot + R - 1) % R);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(K * (R - 1)));       // this row's K DMAs landed
    const double* src = ring + slot * K * 128 + 2 * lane;
    d2 s = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const d2 v = *reinterpret_cast<const d2*>(src + j * 128);
      s.x = s.x + v.x * c[j];
      s.y = s.y + v.y * c[j];
    }
    if (iy < N) __builtin_nontemporal_store(s, reinterpret_cast<d2*>(x + row * N + iy));
    slot = (slot + 1) % R;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
}

__global__ void k_fill(double* v, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    v[i] = 1.0 + double((i * 2654435761LL) & 0xFFFF) * 1e-5;     // nonzero data (zeros clock differently)
}

template <int K>
void run(int64_t N, double* V, double* cv, double* x, int ncu) {
  const int64_t ldv = N * N;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  const double bytes = 8.0 * double(N) * double(N) * (K + 1);
  auto timeit = [&](auto launch, const char* name) {
    for (int i = 0; i < 3; ++i) launch();
    CHK(hipDeviceSynchronize());
    const int reps = 10;
    CHK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("{\"K\": %d, \"mode\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f}\n", K, name, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  const unsigned gx = unsigned(N / (2 * BLOCK));
  for (int rows_per_cu : {4, 8, 16}) {
    const unsigned gy = unsigned(std::max<int64_t>(1, int64_t(ncu) * rows_per_cu / gx));
    char nm[64];
    snprintf(nm, sizeof nm, "vgpr_gy%u", gy);
    timeit([&] { hipLaunchKernelGGL((k_vgpr<K, false>), dim3(gx, gy), dim3(BLOCK), 0, 0, V, ldv, cv, x, N); }, nm);
    snprintf(nm, sizeof nm, "vgpr_pf_gy%u", gy);
    timeit([&] { hipLaunchKernelGGL((k_vgpr<K, true>), dim3(gx, gy), dim3(BLOCK), 0, 0, V, ldv, cv, x, N); }, nm);
  }
  constexpr int R = K <= 4 ? 8 : K <= 8 ? 4 : K <= 12 ? 3 : 2;
  const size_t lds = size_t(4) * R * K * 128 * 8;
  for (int rows_per_cu : {1, 2, 4}) {
    const unsigned gy = unsigned(std::max<int64_t>(1, int64_t(ncu) * rows_per_cu / gx));
    char nm[64];
    snprintf(nm, sizeof nm, "dma_R%d_gy%u", R, gy);
    timeit([&] { hipLaunchKernelGGL((k_dma<K, R, 0>), dim3(gx, gy), dim3(BLOCK), lds, 0, V, ldv, cv, x, N); }, nm);
    snprintf(nm, sizeof nm, "dma_nt_R%d_gy%u", R, gy);
    timeit([&] { hipLaunchKernelGGL((k_dma<K, R, 2>), dim3(gx, gy), dim3(BLOCK), lds, 0, V, ldv, cv, x, N); }, nm);
  }
}

int main() {
  const int64_t N = 8192;
  const int KMAX = 20;
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  double *V, *cv, *x;
  CHK(hipMalloc(&V, sizeof(double) * N * N * KMAX));
  CHK(hipMalloc(&x, sizeof(double) * N * N));
  CHK(hipMalloc(&cv, sizeof(double) * KMAX));
  std::vector<double> h(KMAX, 0.5);
  CHK(hipMemcpy(cv, h.data(), sizeof(double) * KMAX, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, V, N * N * KMAX);
  CHK(hipDeviceSynchronize());
  run<4>(N, V, cv, x, prop.multiProcessorCount);
  run<12>(N, V, cv, x, prop.multiProcessorCount);
  run<20>(N, V, cv, x, prop.multiProcessorCount);
  CHK(hipFree(V));
  CHK(hipFree(x));
  CHK(hipFree(cv));
  return 0;
}
