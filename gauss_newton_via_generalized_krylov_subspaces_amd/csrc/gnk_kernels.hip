// gnk_kernels.hip -- gfx950 (MI355X / CDNA4) kernels + C-ABI for the
// generalized-Krylov Gauss-Newton hot path on the Bratu problem.
//
// Reference algorithm: mariusbaehr/gauss_newton_via_generalized_krylov_subspaces
//   krylow.py:30-73            basis start / x / update (CGS1)         -> gemv, vjp_gemv_t, cgs_update, vec_div
//   gauss_newton_krylow.py:16-36  LAPACK QR of -J@V + q.T@y           -> gram (CholeskyQR2 on fp64 MFMA)
//   armijo_goldstein.py:49-58  sum(res**2) per trial                  -> residual (fused norm)
//   bratu_pde_problem.py:76-96 F(u), CSR Jacobian                     -> matrix-free stencils
//   gauss_newton.py:11-60      scipy cg on A.T A                       -> cg_* kernels
//
// Layout: "slab vectors" of (nrows + 2*GHOST) * N doubles, row-major over the
// grid's x index (flat = jx*N + iy), owned rows at offset GHOST*N (gnk.h).
// Every stencil sum accumulates from 0 in scipy's CSR column order
// (i-N, i-1, i, i+1, i+N); the file is compiled with -ffp-contract=off so
// products and sums round like the reference's sparsetools loops.
//
// Reductions are two-stage and deterministic: per-block partials in the
// context's scratch arena, then one block sums them in block order.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/gnk.h"

#define G GNK_GHOST_ROWS

namespace {

constexpr int BLOCK = 256;
constexpr int MAX_RED_BLOCKS = 1 << 20;  // cap on per-block partials of a reduction
constexpr int PPW_MAX = 10;              // Gram accumulator tiles per wave (pair-split mode)
constexpr size_t SCRATCH_DOUBLES = size_t(16) << 20;   // 128 MiB arena
// offset of the (16 nb)^2 identity in gnk_ctx::ident (nb = 1..4; nb = 5 -> total size)
constexpr int ident_offset(int nb) { return nb == 1 ? 0 : ident_offset(nb - 1) + 256 * (nb - 1) * (nb - 1); }

typedef double d2 __attribute__((ext_vector_type(2)));
// Streaming store of a result vector no kernel of the same launch reads again (the trial point, the new
// basis column, the pending column, the residual): non-temporal, so the written lines do not displace
// what the launch still reads from L2 (the neighbour rows of r, the basis rows of adjacent blocks).
// k_gemv_vjpg at 8192^2: 10-17 % less time than plain stores (profiles/round4/trial_nt_ab.jsonl); k_gemv and
// k_vjp_gemv_t 1-3 % (profiles/round4/nt3_ab.jsonl; k_cgs unchanged, kept plain).
__device__ __forceinline__ void st_nt(double* p, d2 v) { __builtin_nontemporal_store(v, reinterpret_cast<d2*>(p)); }
__device__ __forceinline__ void st_nt(double* p, double v) { __builtin_nontemporal_store(v, p); }
typedef double d4 __attribute__((ext_vector_type(4)));

struct Geo {
  int64_t N;      // row length == number of global rows (square grid)
  int64_t row0;   // global row of the first owned row
  int64_t nrows;  // owned rows
};

// Coefficients of the CSR entries (ref:bratu_pde_problem.py:43-67, 92-96)
struct Coef {
  double hm2;         // h^-2            (= -L off-diagonal)
  double l_off;       // -1 * h^-2
  double l_diag;      // 4 * h^-2
  double dx_diag;     // ALPHA * (-h^-1)
  double dx_up;       // ALPHA * (+h^-1)
  double j_lin_diag;  // l_diag + dx_diag      (L + ALPHA D_x) diagonal
  double j_lin_up;    // l_off + dx_up         (L + ALPHA D_x) at column i+N
  double lam;
  int lam_zero;
};

__device__ __forceinline__ double jdiag(const Coef& c, double u) {
  // diagonal of L + ALPHA D_x + LAMBDA diag(exp u) (ref:bratu_pde_problem.py:92-96)
  return c.lam_zero ? c.j_lin_diag : c.j_lin_diag + c.lam * exp(u);
}

// J v at one point: J = -(...), CSR row order i-N, i-1, i, i+1, i+N
__device__ __forceinline__ double jvp_pt(const Coef& c, double d, double vn, double vw, bool hw,
                                         double vc, double ve, bool he, double vs) {
  double s = 0.0 + c.hm2 * vn;
  if (hw) s = s + c.hm2 * vw;
  s = s + (-d) * vc;
  if (he) s = s + c.hm2 * ve;
  s = s + (-c.j_lin_up) * vs;
  return s;
}

// J^T w at one point: csc_matvec order (source rows ascending)
__device__ __forceinline__ double vjp_pt(const Coef& c, double d, double wn, double ww, bool hw,
                                         double wc, double we, bool he, double ws) {
  double s = 0.0 + (-c.j_lin_up) * wn;
  if (hw) s = s + c.hm2 * ww;
  s = s + (-d) * wc;
  if (he) s = s + c.hm2 * we;
  s = s + c.hm2 * ws;
  return s;
}

// pde_operator(x) at one point: (L x + (ALPHA D_x) x) + LAMBDA exp(x)
__device__ __forceinline__ double fwd_pt(const Coef& c, double xn, double xw, bool hw, double xc,
                                         double xe, bool he, double xs) {
  double l = 0.0 + c.l_off * xn;
  if (hw) l = l + c.l_off * xw;
  l = l + c.l_diag * xc;
  if (he) l = l + c.l_off * xe;
  l = l + c.l_off * xs;
  double dx = 0.0 + c.dx_diag * xc;
  dx = dx + c.dx_up * xs;
  double f = l + dx;
  if (!c.lam_zero) f = f + c.lam * exp(xc);
  return f;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double nan_max(double a, double b) {
  // max that propagates NaN (np.allclose never calls a NaN close)
  return (b > a || b != b) ? b : a;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = nan_max(v, __shfl_xor(v, o));
  return v;
}

// block-wide sum of `n` per-thread values, result written by thread 0..n-1 into out[0..n)
template <int NV>
__device__ __forceinline__ void block_sum_store(double (&v)[NV], int n, double* out, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    if (j < n) {
      double s = wave_sum(v[j]);
      if (lane == 0) sh[wave * NV + j] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x < n) {
    double s = sh[threadIdx.x];
    for (int w = 1; w < BLOCK / 64; ++w) s += sh[w * NV + threadIdx.x];
    out[threadIdx.x] = s;
  }
}

// ---- compensated sums (Ogita-Rump-Oishi Sum2 / Dot2): a value is carried as s + c, every addition
// keeps its rounding error (TwoSum) and every product its FMA-exact error (TwoProduct), so a dot
// product is as accurate as if accumulated in twice the working precision and rounded once.  Used
// for the CG scalars (p.q, r.r, r.z, ||b||), whose exact rounding decides scipy's stopping test
// ||r|| < rtol ||b|| (ref:gauss_newton.py:36-58 via scipy iterative.py:397): the reference's own
// OpenBLAS dot is within a few ulps of the exactly rounded value, and so is this one, whatever the
// block / wave / rank partition.  (-ffp-contract=off keeps TwoSum intact.)
__device__ __forceinline__ void comp_add(double& s, double& c, double v) {
  const double t = s + v;
  const double bp = t - s;
  c += (s - (t - bp)) + (v - bp);
  s = t;
}
__device__ __forceinline__ void comp_dot(double& s, double& c, double a, double b) {
  const double pr = a * b;
  c += fma(a, b, -pr);
  comp_add(s, c, pr);
}
__device__ __forceinline__ void comp_merge(double& s, double& c, double s2, double c2) {
  comp_add(s, c, s2);
  c += c2;
}
__device__ __forceinline__ void wave_sum2(double& s, double& c) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double s2 = __shfl_xor(s, o), c2 = __shfl_xor(c, o);
    comp_merge(s, c, s2, c2);
  }
}
// block-wide compensated sums of n per-thread (s, c) pairs -> out[2j] = s_j, out[2j + 1] = c_j
template <int NV>
__device__ __forceinline__ void block_sum2_store(double (&s)[NV], double (&c)[NV], int n, double* out, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    if (j < n) {
      wave_sum2(s[j], c[j]);
      if (lane == 0) {
        sh[(wave * NV + j) * 2] = s[j];
        sh[(wave * NV + j) * 2 + 1] = c[j];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < n) {
    const int j = threadIdx.x;
    double a = sh[2 * j], b = sh[2 * j + 1];
    for (int w = 1; w < BLOCK / 64; ++w) comp_merge(a, b, sh[(w * NV + j) * 2], sh[(w * NV + j) * 2 + 1]);
    out[2 * j] = a;
    out[2 * j + 1] = b;
  }
}

// ---------------------------------------------------------------- row-tiled launch geometry
// grid.x covers one row (VEC elements per thread), grid.y strides over rows.
struct RowLaunch {
  dim3 grid;
  int64_t lr0, nlr;  // local row range [lr0, lr0 + nlr)
};

// Element loop helper: for local row lr and element iy of a row.  grid.x strides along the row:
// the Bratu launches (rows()) cover a whole row with grid.x (one pass), the flat launches of the
// generic path (flat_rows(), one "row" of n) may cap grid.x, and then every thread walks the row.
#define ROW_LOOP_BEGIN(VEC)                                                                      \
  const int64_t N = geo.N;                                                                       \
  for (int64_t lr = lr0 + blockIdx.y; lr < lr0 + nlr; lr += gridDim.y) {                         \
    for (int64_t iy = (int64_t(blockIdx.x) * BLOCK + threadIdx.x) * (VEC); iy < N;               \
         iy += int64_t(gridDim.x) * BLOCK * (VEC)) {                                             \
      const int64_t li = lr * N + iy;

#define ROW_LOOP_END }}

// Row loop of the persistent reduction kernels with segments (gnk_set_segments): grid.z = nseg + 1 slices,
// slice z < nseg the owned rows of segment z (block row y taking rows y, y + gridDim.y, .. counted from the
// segment's first row: a block's rows in a segment do not depend on where the slab starts), slice nseg the
// rest of [lr0, lr0 + nlr) (ghost rows, no partial contributions).  seg == 0: one slice, [lr0, lr0 + nlr) as
// ROW_LOOP.  One loop around one copy of the body, as ROW_LOOP (a loop over segments with a partial store
// per segment in the kernel raised the trial kernel's VGPRs to 256).
#define ZSEG_ROW_LOOP_BEGIN(VEC)                                                                        \
  const int64_t N = geo.N;                                                                             \
  const int zs = blockIdx.z;                                                                           \
  const bool ghost_slice = seg > 0 && zs == nseg;                                                      \
  const int64_t gbelow = max(int64_t(0), G - lr0);             /* ghost rows before the owned ones */  \
  const int64_t za = seg == 0 ? lr0 : (ghost_slice ? lr0 : G + int64_t(zs) * seg);                     \
  const int64_t zcnt = seg == 0 ? nlr : (ghost_slice ? nlr - geo.nrows : seg);                         \
  for (int64_t t = blockIdx.y; t < zcnt; t += gridDim.y) {                                             \
    const int64_t lr = (ghost_slice && t >= gbelow) ? G + geo.nrows + (t - gbelow) : za + t;           \
    for (int64_t iy = (int64_t(blockIdx.x) * BLOCK + threadIdx.x) * (VEC); iy < N;                     \
         iy += int64_t(gridDim.x) * BLOCK * (VEC)) {                                                   \
      const int64_t li = lr * N + iy;

#define ZSEG_ROW_LOOP_END }}

// ---------------------------------------------------------------- in-row neighbours across lanes
// Lane l <- lane l - 1 / l + 1 of the wave: DPP wave_shr:1 / wave_shl:1 (gfx9), two 32-bit VALU moves per
// double instead of the two ds_bpermute LDS round trips __shfl_up / __shfl_down compile to (the k = 8, 9
// VALU Gram pass 6-9 % faster, bit-identical: profiles/round5/lane_dpp_ab.jsonl).  Lanes 0 / 63 get 0:
// every caller replaces them with the strip's outer neighbour.  Used by the VALU Gram passes and the row-marching
// CG normal matvec.  (Round 5 kept them out of the persistent trial kernels, whose grid then followed the
// occupancy; since round 6 every grid carrying partial sums is a fixed table, so a VGPR change no longer moves
// any reduction's bits -- DESIGN.md §7d, tests/test_gpu_decomp.py.)
typedef unsigned int lane_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double lane_prev(double v) {
  const lane_u2 b = __builtin_bit_cast(lane_u2, v);
  lane_u2 o;
  o.x = unsigned(__builtin_amdgcn_mov_dpp(int(b.x), 0x138, 0xf, 0xf, true));
  o.y = unsigned(__builtin_amdgcn_mov_dpp(int(b.y), 0x138, 0xf, 0xf, true));
  return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double lane_next(double v) {
  const lane_u2 b = __builtin_bit_cast(lane_u2, v);
  lane_u2 o;
  o.x = unsigned(__builtin_amdgcn_mov_dpp(int(b.x), 0x130, 0xf, 0xf, true));
  o.y = unsigned(__builtin_amdgcn_mov_dpp(int(b.y), 0x130, 0xf, 0xf, true));
  return __builtin_bit_cast(double, o);
}

// ---------------------------------------------------------------- operator kernels
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_jvp(const double* __restrict__ u, const double* __restrict__ v,
                                               double* __restrict__ out, Geo geo, Coef c, int64_t lr0,
                                               int64_t nlr, int transpose) {
  const int lane = threadIdx.x & 63;
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    // two points per lane: 16-B loads of u, v and the rows above/below; the in-row
    // neighbours come from the adjacent lanes (lane 0 / 63 load their outer one)
    const d2 uc = *reinterpret_cast<const d2*>(u + li);
    const d2 vc = *reinterpret_cast<const d2*>(v + li);
    const d2 vn = *reinterpret_cast<const d2*>(v + li - N);
    const d2 vs = *reinterpret_cast<const d2*>(v + li + N);
    const bool hw = iy > 0, he = iy + 2 < N;
    double vw = __shfl_up(vc.y, 1);
    double ve = __shfl_down(vc.x, 1);
    if (lane == 0) vw = hw ? v[li - 1] : 0.0;
    if (lane == 63 || iy + 2 >= N) ve = he ? v[li + 2] : 0.0;
    const double d0 = jdiag(c, uc.x), d1 = jdiag(c, uc.y);
    d2 o;
    if (transpose) {
      o.x = vjp_pt(c, d0, vn.x, vw, hw, vc.x, vc.y, true, vs.x);
      o.y = vjp_pt(c, d1, vn.y, vc.x, true, vc.y, ve, he, vs.y);
    } else {
      o.x = jvp_pt(c, d0, vn.x, vw, hw, vc.x, vc.y, true, vs.x);
      o.y = jvp_pt(c, d1, vn.y, vc.x, true, vc.y, ve, he, vs.y);
    }
    *reinterpret_cast<d2*>(out + li) = o;
  } else {
    for (int q = 0; q < VEC; ++q) {
      const int64_t i = li + q;
      const int64_t y = iy + q;
      if (y >= N) break;
      const bool hw = y > 0, he = y < N - 1;
      const double d = jdiag(c, u[i]);
      const double vn = v[i - N], vs = v[i + N], vc = v[i];
      const double vw = hw ? v[i - 1] : 0.0, ve = he ? v[i + 1] : 0.0;
      out[i] = transpose ? vjp_pt(c, d, vn, vw, hw, vc, ve, he, vs) : jvp_pt(c, d, vn, vw, hw, vc, ve, he, vs);
    }
  }
  ROW_LOOP_END
}

template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_forward(const double* __restrict__ x, const double* __restrict__ y,
                                                   double* __restrict__ out, Geo geo, Coef c, int64_t lr0,
                                                   int64_t nlr, double* __restrict__ partial) {
  // out = pde_operator(x) (y == nullptr) or y - pde_operator(x); partial: sum out^2 over owned rows
  __shared__ double sh[BLOCK / 64];
  const int lane = threadIdx.x & 63;
  double acc[1] = {0.0};
  ROW_LOOP_BEGIN(VEC)
  const bool owned = lr >= G && lr < G + geo.nrows;
  if (VEC == 2 && iy + 1 < N) {
    const d2 xc = *reinterpret_cast<const d2*>(x + li);
    const d2 xn = *reinterpret_cast<const d2*>(x + li - N);
    const d2 xs = *reinterpret_cast<const d2*>(x + li + N);
    const bool hw = iy > 0, he = iy + 2 < N;
    double xw = __shfl_up(xc.y, 1);
    double xe = __shfl_down(xc.x, 1);
    if (lane == 0) xw = hw ? x[li - 1] : 0.0;
    if (lane == 63 || iy + 2 >= N) xe = he ? x[li + 2] : 0.0;
    d2 f;
    f.x = fwd_pt(c, xn.x, xw, hw, xc.x, xc.y, true, xs.x);
    f.y = fwd_pt(c, xn.y, xc.x, true, xc.y, xe, he, xs.y);
    if (y) {
      const d2 yy = *reinterpret_cast<const d2*>(y + li);
      f.x = yy.x - f.x;
      f.y = yy.y - f.y;
    }
    *reinterpret_cast<d2*>(out + li) = f;
    if (owned) {
      acc[0] += f.x * f.x;
      acc[0] += f.y * f.y;
    }
  } else {
    for (int q = 0; q < VEC; ++q) {
      const int64_t i = li + q;
      const int64_t yy = iy + q;
      if (yy >= N) break;
      const bool hw = yy > 0, he = yy < N - 1;
      const double xw = hw ? x[i - 1] : 0.0, xe = he ? x[i + 1] : 0.0;
      const double f = fwd_pt(c, x[i - N], xw, hw, x[i], xe, he, x[i + N]);
      const double rr = y ? y[i] - f : f;
      out[i] = rr;
      if (owned) acc[0] += rr * rr;
    }
  }
  ROW_LOOP_END
  if (partial) block_sum_store<1>(acc, 1, partial + (blockIdx.y * gridDim.x + blockIdx.x), sh);
}

// Two grid rows per pass (rows lr, lr + 1; VEC 2 and N % 512 == 0, so every lane of every block holds
// two points of the row -- no lanes past its end): the centre and south rows of the stencil vector serve both output rows, 4 row loads
// per 2 output rows instead of 6.  The per-point arithmetic is k_jvp's / k_forward's, bit for bit.
// 8192^2 JVP 0.319 -> 0.271 ms (5.05 -> 5.94 TB/s), 16384^2 5.6 -> 6.05 TB/s
// (profiles/round3/jvp2_ab.jsonl).  Launched with gridDim.y = ceil(nlr / 2): one pass per block.
constexpr int ROWS2_ALIGN = 2 * BLOCK;

// J(u) v (TR false) / J(u)^T w (TR true)
template <bool TR>
__global__ __launch_bounds__(BLOCK) void k_jvp2(const double* __restrict__ u, const double* __restrict__ v,
                                                double* __restrict__ out, Geo geo, Coef c, int64_t lr0, int64_t nlr) {
  const int lane = threadIdx.x & 63;
  const int64_t N = geo.N;
  const int64_t iy = (int64_t(blockIdx.x) * BLOCK + threadIdx.x) * 2;
  const bool hw = iy > 0, he = iy + 2 < N;
  for (int64_t p = blockIdx.y; 2 * p < nlr; p += gridDim.y) {
    const int64_t lr = lr0 + 2 * p;
    const bool two = 2 * p + 1 < nlr;               // block-uniform
    const int64_t li = lr * N + iy;
    const d2 vn = *reinterpret_cast<const d2*>(v + li - N);
    const d2 vc = *reinterpret_cast<const d2*>(v + li);
    const d2 vs = *reinterpret_cast<const d2*>(v + li + N);
    const d2 u0 = *reinterpret_cast<const d2*>(u + li);
    d2 vss = {0.0, 0.0}, u1 = {0.0, 0.0};
    if (two) {
      vss = *reinterpret_cast<const d2*>(v + li + 2 * N);
      u1 = *reinterpret_cast<const d2*>(u + li + N);
    }
    double vw0 = __shfl_up(vc.y, 1), ve0 = __shfl_down(vc.x, 1);
    double vw1 = __shfl_up(vs.y, 1), ve1 = __shfl_down(vs.x, 1);
    if (lane == 0) {
      vw0 = hw ? v[li - 1] : 0.0;
      vw1 = hw ? v[li + N - 1] : 0.0;
    }
    if (lane == 63) {
      ve0 = he ? v[li + 2] : 0.0;
      ve1 = he ? v[li + N + 2] : 0.0;
    }
    const double d00 = jdiag(c, u0.x), d01 = jdiag(c, u0.y);
    d2 o;
    if (TR) {
      o.x = vjp_pt(c, d00, vn.x, vw0, hw, vc.x, vc.y, true, vs.x);
      o.y = vjp_pt(c, d01, vn.y, vc.x, true, vc.y, ve0, he, vs.y);
    } else {
      o.x = jvp_pt(c, d00, vn.x, vw0, hw, vc.x, vc.y, true, vs.x);
      o.y = jvp_pt(c, d01, vn.y, vc.x, true, vc.y, ve0, he, vs.y);
    }
    *reinterpret_cast<d2*>(out + li) = o;
    if (two) {
      const double d10 = jdiag(c, u1.x), d11 = jdiag(c, u1.y);
      if (TR) {
        o.x = vjp_pt(c, d10, vc.x, vw1, hw, vs.x, vs.y, true, vss.x);
        o.y = vjp_pt(c, d11, vc.y, vs.x, true, vs.y, ve1, he, vss.y);
      } else {
        o.x = jvp_pt(c, d10, vc.x, vw1, hw, vs.x, vs.y, true, vss.x);
        o.y = jvp_pt(c, d11, vc.y, vs.x, true, vs.y, ve1, he, vss.y);
      }
      *reinterpret_cast<d2*>(out + li + N) = o;
    }
  }
}

// out = pde_operator(x) (y == nullptr) or y - pde_operator(x).  partial (residual): the sum of out^2 over
// each owned row's 512-point segment at [row offset * gridDim.x + blockIdx.x] -- exactly k_forward's
// partials when that kernel runs one row per block (same per-thread order, same block reduction)
__global__ __launch_bounds__(BLOCK) void k_forward2(const double* __restrict__ x, const double* __restrict__ y,
                                                    double* __restrict__ out, Geo geo, Coef c, int64_t lr0,
                                                    int64_t nlr, double* __restrict__ partial) {
  __shared__ double sh[2][BLOCK / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t N = geo.N;
  const int64_t iy = (int64_t(blockIdx.x) * BLOCK + threadIdx.x) * 2;
  const bool hw = iy > 0, he = iy + 2 < N;
  for (int64_t p = blockIdx.y; 2 * p < nlr; p += gridDim.y) {
    const int64_t lr = lr0 + 2 * p;
    const bool two = 2 * p + 1 < nlr;               // block-uniform
    const int64_t li = lr * N + iy;
    const d2 xn = *reinterpret_cast<const d2*>(x + li - N);
    const d2 xc = *reinterpret_cast<const d2*>(x + li);
    const d2 xs = *reinterpret_cast<const d2*>(x + li + N);
    d2 xss = {0.0, 0.0};
    if (two) xss = *reinterpret_cast<const d2*>(x + li + 2 * N);
    double xw0 = __shfl_up(xc.y, 1), xe0 = __shfl_down(xc.x, 1);
    double xw1 = __shfl_up(xs.y, 1), xe1 = __shfl_down(xs.x, 1);
    if (lane == 0) {
      xw0 = hw ? x[li - 1] : 0.0;
      xw1 = hw ? x[li + N - 1] : 0.0;
    }
    if (lane == 63) {
      xe0 = he ? x[li + 2] : 0.0;
      xe1 = he ? x[li + N + 2] : 0.0;
    }
    double acc0 = 0.0, acc1 = 0.0;
    d2 f;
    f.x = fwd_pt(c, xn.x, xw0, hw, xc.x, xc.y, true, xs.x);
    f.y = fwd_pt(c, xn.y, xc.x, true, xc.y, xe0, he, xs.y);
    if (y) {
      const d2 yy = *reinterpret_cast<const d2*>(y + li);
      f.x = yy.x - f.x;
      f.y = yy.y - f.y;
    }
    *reinterpret_cast<d2*>(out + li) = f;
    if (lr >= G && lr < G + geo.nrows) {
      acc0 += f.x * f.x;
      acc0 += f.y * f.y;
    }
    if (two) {
      f.x = fwd_pt(c, xc.x, xw1, hw, xs.x, xs.y, true, xss.x);
      f.y = fwd_pt(c, xc.y, xs.x, true, xs.y, xe1, he, xss.y);
      if (y) {
        const d2 yy = *reinterpret_cast<const d2*>(y + li + N);
        f.x = yy.x - f.x;
        f.y = yy.y - f.y;
      }
      *reinterpret_cast<d2*>(out + li + N) = f;
      if (lr + 1 >= G && lr + 1 < G + geo.nrows) {
        acc1 += f.x * f.x;
        acc1 += f.y * f.y;
      }
    }
    if (partial) {
      const double s0 = wave_sum(acc0), s1 = wave_sum(acc1);
      if (lane == 0) {
        sh[0][wave] = s0;
        sh[1][wave] = s1;
      }
      __syncthreads();
      if (threadIdx.x < (two ? 2 : 1)) {
        const int q = threadIdx.x;
        double t = sh[q][0];
        for (int w = 1; w < BLOCK / 64; ++w) t += sh[q][w];
        partial[(2 * p + q) * int64_t(gridDim.x) + blockIdx.x] = t;
      }
      __syncthreads();
    }
  }
}

template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_diag_jtj(const double* __restrict__ u, double* __restrict__ out,
                                                    Geo geo, Coef c, int64_t lr0, int64_t nlr, int recip) {
  ROW_LOOP_BEGIN(VEC)
  const int64_t grow = geo.row0 + (lr - G);
#pragma unroll
  for (int q = 0; q < VEC; ++q) {
    const int64_t i = li + q;
    const int64_t yy = iy + q;
    if (yy >= N) break;
    const double d = jdiag(c, u[i]);
    const double o2 = c.l_off * c.l_off;
    const double up = grow > 0 ? c.j_lin_up * c.j_lin_up : 0.0;
    const double west = yy > 0 ? o2 : 0.0;
    const double east = yy < N - 1 ? o2 : 0.0;
    const double south = grow < N - 1 ? o2 : 0.0;
    const double v = (((up + west) + d * d) + east) + south;
    out[i] = recip ? 1.0 / v : v;
  }
  ROW_LOOP_END
}

// ---------------------------------------------------------------- basis kernels
// x = V[:, :k] @ c
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_gemv(const double* __restrict__ V, int64_t ldv, int k,
                                                const double* __restrict__ cvec, double* __restrict__ x,
                                                Geo geo, int64_t lr0, int64_t nlr) {
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    d2 acc = {0.0, 0.0};
    for (int j = 0; j < k; ++j) {
      const d2 vv = *reinterpret_cast<const d2*>(V + j * ldv + li);
      const double cj = cvec[j];
      acc.x = acc.x + vv.x * cj;
      acc.y = acc.y + vv.y * cj;
    }
    st_nt(x + li, acc);
  } else {
    for (int q = 0; q < VEC && iy + q < N; ++q) {
      double acc = 0.0;
      for (int j = 0; j < k; ++j) acc = acc + V[j * ldv + li + q] * cvec[j];
      x[li + q] = acc;
    }
  }
  ROW_LOOP_END
}

// block-wide {sum, NaN-propagating max} -> partial[2 blk], partial[2 blk + 1]
__device__ __forceinline__ void block_sum_max_store(double ss, double mx, double* __restrict__ partial) {
  __shared__ double shm[BLOCK / 64][2];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  ss = wave_sum(ss);
  mx = wave_max(mx);
  if (lane == 0) { shm[wave][0] = ss; shm[wave][1] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = shm[0][0], b = shm[0][1];
    for (int w = 1; w < BLOCK / 64; ++w) { a += shm[w][0]; b = nan_max(b, shm[w][1]); }
    const size_t blk = blockIdx.y * gridDim.x + blockIdx.x;
    partial[2 * blk] = a;
    partial[2 * blk + 1] = b;
  }
}

// Trial point with the pending basis column materialised (deferred CGS of krylow.py:64):
//   w = g - V[:, :k] @ hh        in place over column k (= g), whole slab, the rounding of k_cgs;
//   x = V[:, :k] @ c[:k] + w c[k]   the rounding of k_gemv over k + 1 columns;
//   partial {sum w^2, max |w|} over owned rows (the norm and breakdown test of krylow.py:66, 71).
// Column k is read and written only through `w` (never through V).
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_gemv_p(const double* __restrict__ V, int64_t ldv, int k,
                                                  const double* __restrict__ cvec, const double* __restrict__ hh,
                                                  double* __restrict__ w, double* __restrict__ x, Geo geo,
                                                  int64_t lr0, int64_t nlr, double* __restrict__ partial,
                                                  int64_t seg, int nseg) {
  double ss = 0.0, mx = 0.0;
  const double ck = cvec[k];
  ZSEG_ROW_LOOP_BEGIN(VEC)
  const bool owned = lr >= G && lr < G + geo.nrows;       // block-uniform
  if (VEC == 2 && iy + 1 < N) {
    d2 acc = {0.0, 0.0}, s = {0.0, 0.0};
    for (int j = 0; j < k; ++j) {
      const d2 vv = *reinterpret_cast<const d2*>(V + j * ldv + li);
      const double cj = cvec[j], hj = hh[j];
      acc.x = acc.x + vv.x * cj;
      acc.y = acc.y + vv.y * cj;
      s.x = s.x + vv.x * hj;
      s.y = s.y + vv.y * hj;
    }
    d2 ww = *reinterpret_cast<const d2*>(w + li);
    ww.x = ww.x - s.x;
    ww.y = ww.y - s.y;
    st_nt(w + li, ww);
    acc.x = acc.x + ww.x * ck;
    acc.y = acc.y + ww.y * ck;
    st_nt(x + li, acc);
    if (owned) {
      ss += ww.x * ww.x;
      ss += ww.y * ww.y;
      mx = nan_max(mx, fabs(ww.x));
      mx = nan_max(mx, fabs(ww.y));
    }
  } else {
    for (int q = 0; q < VEC && iy + q < N; ++q) {
      double acc = 0.0, s = 0.0;
      for (int j = 0; j < k; ++j) {
        const double vv = V[j * ldv + li + q];
        acc = acc + vv * cvec[j];
        s = s + vv * hh[j];
      }
      const double wi = w[li + q] - s;
      st_nt(w + li + q, wi);
      st_nt(x + li + q, acc + wi * ck);
      if (owned) {
        ss += wi * wi;
        mx = nan_max(mx, fabs(wi));
      }
    }
  }
  ZSEG_ROW_LOOP_END
  block_sum_max_store(ss, mx, partial + 2 * size_t(blockIdx.z) * gridDim.x * gridDim.y);
}

// g = -(J^T r) on owned rows (chunk 0 stores it), h[j0 + j] partial = V_j . g.
// KCT columns per chunk (compile time): every V load is unconditional (clamped column),
// surplus accumulators are discarded by the block reduction (no loads under a branch).
// GREAD: g is read back (stored by an earlier launch of the same row decomposition) instead of
// recomputed from u and r -- the wide-basis split of gnk_vjp_gemv_t; the same products in the same
// order, so the same partials.
template <int VEC, int KCT, bool GREAD = false>
__global__ __launch_bounds__(BLOCK) void k_vjp_gemv_t(const double* __restrict__ u, const double* __restrict__ r,
                                                      const double* __restrict__ V, int64_t ldv, int k,
                                                      double* __restrict__ g, Geo geo, Coef c, int64_t lr0,
                                                      int64_t nlr, double* __restrict__ partial, int z0) {
  __shared__ double sh[(BLOCK / 64) * KCT];
  const int lane = threadIdx.x & 63;
  const int zc = z0 + int(blockIdx.z);              // column chunk (launches may cover a range of chunks)
  const int j0 = zc * KCT;
  const int kc = max(0, min(KCT, k - j0));
  const int jmax = max(k - 1, 0);
  double acc[KCT];
#pragma unroll
  for (int j = 0; j < KCT; ++j) acc[j] = 0.0;
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    double g0, g1;
    if constexpr (GREAD) {
      const d2 gg = *reinterpret_cast<const d2*>(g + li);
      g0 = gg.x;
      g1 = gg.y;
    } else {
      const d2 uc = *reinterpret_cast<const d2*>(u + li);
      const d2 rc = *reinterpret_cast<const d2*>(r + li);
      const d2 rn = *reinterpret_cast<const d2*>(r + li - N);
      const d2 rs = *reinterpret_cast<const d2*>(r + li + N);
      const bool hw = iy > 0, he = iy + 2 < N;
      double rw = __shfl_up(rc.y, 1);
      double re = __shfl_down(rc.x, 1);
      if (lane == 0) rw = hw ? r[li - 1] : 0.0;
      if (lane == 63 || iy + 2 >= N) re = he ? r[li + 2] : 0.0;
      g0 = -vjp_pt(c, jdiag(c, uc.x), rn.x, rw, hw, rc.x, rc.y, true, rs.x);
      g1 = -vjp_pt(c, jdiag(c, uc.y), rn.y, rc.x, true, rc.y, re, he, rs.y);
      if (zc == 0) st_nt(g + li, d2{g0, g1});
    }
    if (k > 0) {
#pragma unroll
      for (int j = 0; j < KCT; ++j) {
        const d2 vv = *reinterpret_cast<const d2*>(V + min(j0 + j, jmax) * ldv + li);
        acc[j] = acc[j] + vv.x * g0;
        acc[j] = acc[j] + vv.y * g1;
      }
    }
  } else {
    for (int q = 0; q < VEC; ++q) {
      const int64_t i = li + q;
      const int64_t yy = iy + q;
      if (yy >= N) break;
      double gi;
      if constexpr (GREAD) {
        gi = g[i];
      } else {
        const bool hw = yy > 0, he = yy < N - 1;
        const double d = jdiag(c, u[i]);
        const double rw = hw ? r[i - 1] : 0.0, re = he ? r[i + 1] : 0.0;
        gi = -vjp_pt(c, d, r[i - N], rw, hw, r[i], re, he, r[i + N]);
        if (zc == 0) g[i] = gi;
      }
      if (k > 0) {
#pragma unroll
        for (int j = 0; j < KCT; ++j) acc[j] = acc[j] + V[min(j0 + j, jmax) * ldv + i] * gi;
      }
    }
  }
  ROW_LOOP_END
  const int nblk = gridDim.x * gridDim.y;
  block_sum_store<KCT>(acc, kc, partial + (size_t(blockIdx.z) * nblk + blockIdx.y * gridDim.x + blockIdx.x) * KCT, sh);
}

// Fused trial step + basis-update products (version res_old, first Armijo trial):
//   x = V[:, :k] @ c on the whole slab (same arithmetic as k_gemv), and on owned rows
//   g = -(J(x)^T r) (J at the trial point: only x_i enters the diagonal) and partial h = V^T g,
// from ONE read of V (k_gemv + k_vjp_gemv_t read it twice and read u = x back).
// One chunk of KCT >= k columns; surplus columns are clamped loads with c = 0 and discarded
// partials (no loads under a branch).
// PEND: column k is the pending (raw) basis column g_k of the deferred CGS; it is materialised
// in place first, w = g_k - V[:, :k] @ hh (the rounding of k_cgs: hh_j = 0 past k adds zeros),
// and then enters x and h as column k (k + 1 columns, h partials for all of them); spart gets
// {sum w^2, max |w|} over owned rows.
template <int VEC, int KCT, bool PEND>
__global__ __launch_bounds__(BLOCK) void k_gemv_vjpg(const double* __restrict__ V, int64_t ldv, int k,
                                                     const double* __restrict__ cvec, const double* __restrict__ hh,
                                                     double* __restrict__ wcol, const double* __restrict__ r,
                                                     double* __restrict__ x, double* __restrict__ g, Geo geo, Coef c,
                                                     int64_t lr0, int64_t nlr, double* __restrict__ partial,
                                                     double* __restrict__ spart, int64_t seg, int nseg) {
  __shared__ double sh[(BLOCK / 64) * KCT];
  __shared__ __attribute__((aligned(16))) double cl[2 * KCT];   // [c_0 .. c_{KCT-1} | hh_0 .. hh_{KCT-1}]
  const int lane = threadIdx.x & 63;
  const int kk = PEND ? k + 1 : k;                  // columns entering x and h
  const int jmax = PEND ? k - 1 : kk - 1;           // last column read through V (>= 0: k >= 1)
  // The coefficients live in LDS and are read per row (broadcast reads): held in SGPRs for the whole
  // kernel they spilled (200+ SGPRs at KCT = 16, one v_readlane per use)
  for (int j = threadIdx.x; j < 2 * KCT; j += BLOCK)
    cl[j] = j < KCT ? (j < kk ? cvec[j] : 0.0) : ((PEND && j - KCT < k) ? hh[j - KCT] : 0.0);
  __syncthreads();
  double acc[KCT];
#pragma unroll
  for (int j = 0; j < KCT; ++j) acc[j] = 0.0;
  double ss = 0.0, mx = 0.0;
  ZSEG_ROW_LOOP_BEGIN(VEC)
  const bool owned = lr >= G && lr < G + geo.nrows;       // block-uniform
  if (VEC == 2 && iy + 1 < N) {
    // column j of this grid row: a wave-uniform base (SGPRs) + this lane's 32-bit byte offset
    const uint32_t boff = uint32_t(iy) * uint32_t(sizeof(double));
    d2 vv[KCT];
#pragma unroll
    for (int j = 0; j < KCT; ++j) {
      const char* rowj = reinterpret_cast<const char*>(V + (int64_t(min(j, jmax)) * ldv + lr * N));
      vv[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(rowj + boff));   // streamed once
    }
    int z = 0;
    asm volatile("" : "+s"(z));                     // opaque 0: the LDS reads stay in the row loop
    const double* cz = cl + z;
    if (PEND) {
      d2 s = {0.0, 0.0};
#pragma unroll
      for (int j = 0; j < KCT; ++j) {
        const double hj = cz[KCT + j];
        s.x = s.x + vv[j].x * hj;
        s.y = s.y + vv[j].y * hj;
      }
      d2 ww = *reinterpret_cast<const d2*>(wcol + li);
      ww.x = ww.x - s.x;
      ww.y = ww.y - s.y;
      st_nt(wcol + li, ww);
#pragma unroll
      for (int j = 0; j < KCT; ++j)
        if (j == k) vv[j] = ww;
      if (owned) {
        ss += ww.x * ww.x;
        ss += ww.y * ww.y;
        mx = nan_max(mx, fabs(ww.x));
        mx = nan_max(mx, fabs(ww.y));
      }
    }
    d2 xs = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < KCT; ++j) {
      // the rounding of k_gemv: acc + v_j * c_j in column order (c_j = 0 past k adds a zero)
      const double cj = cz[j];
      xs.x = xs.x + vv[j].x * cj;
      xs.y = xs.y + vv[j].y * cj;
    }
    st_nt(x + li, xs);
    if (owned) {
      const d2 rc = *reinterpret_cast<const d2*>(r + li);
      const d2 rn = *reinterpret_cast<const d2*>(r + li - N);
      const d2 rs = *reinterpret_cast<const d2*>(r + li + N);
      const bool hw = iy > 0, he = iy + 2 < N;
      double rw = __shfl_up(rc.y, 1);
      double re = __shfl_down(rc.x, 1);
      if (lane == 0) rw = hw ? r[li - 1] : 0.0;
      if (lane == 63 || iy + 2 >= N) re = he ? r[li + 2] : 0.0;
      const double g0 = -vjp_pt(c, jdiag(c, xs.x), rn.x, rw, hw, rc.x, rc.y, true, rs.x);
      const double g1 = -vjp_pt(c, jdiag(c, xs.y), rn.y, rc.x, true, rc.y, re, he, rs.y);
      st_nt(g + li, d2{g0, g1});
#pragma unroll
      for (int j = 0; j < KCT; ++j) {
        acc[j] = acc[j] + vv[j].x * g0;
        acc[j] = acc[j] + vv[j].y * g1;
      }
    }
  } else {
    for (int q = 0; q < VEC; ++q) {
      const int64_t i = li + q;
      const int64_t yy = iy + q;
      if (yy >= N) break;
      double vv[KCT];
#pragma unroll
      for (int j = 0; j < KCT; ++j) vv[j] = V[min(j, jmax) * ldv + i];
      if (PEND) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < KCT; ++j) s = s + vv[j] * cl[KCT + j];
        const double wi = wcol[i] - s;
        st_nt(wcol + i, wi);
#pragma unroll
        for (int j = 0; j < KCT; ++j)
          if (j == k) vv[j] = wi;
        if (owned) {
          ss += wi * wi;
          mx = nan_max(mx, fabs(wi));
        }
      }
      double xs = 0.0;
#pragma unroll
      for (int j = 0; j < KCT; ++j) xs = xs + vv[j] * cl[j];
      st_nt(x + i, xs);
      if (owned) {
        const bool hw = yy > 0, he = yy < N - 1;
        const double rw = hw ? r[i - 1] : 0.0, re = he ? r[i + 1] : 0.0;
        const double gi = -vjp_pt(c, jdiag(c, xs), r[i - N], rw, hw, r[i], re, he, r[i + N]);
        st_nt(g + i, gi);
#pragma unroll
        for (int j = 0; j < KCT; ++j) acc[j] = acc[j] + vv[j] * gi;
      }
    }
  }
  ZSEG_ROW_LOOP_END
  // slice z's partials at z * nblk + blk (segments; z = 0 otherwise)
  const size_t zb = size_t(blockIdx.z) * gridDim.x * gridDim.y;
  block_sum_store<KCT>(acc, kk, partial + (zb + size_t(blockIdx.y) * gridDim.x + blockIdx.x) * KCT, sh);
  if (PEND) block_sum_max_store(ss, mx, spart + 2 * zb);
}

// ---------------------------------------------------------------- wide fused first trial (25..208 columns)
// k_gemv_vjpg for bases too wide to hold a point's basis row in VGPRs (C5 grows the basis to 100 columns, 200 on
// 8 GPUs): the same products -- the pending column w = g - V hh materialised in place, x = V c, g = -J(x)^T r on
// owned rows, h = V^T g and {sum w^2, max |w|} over owned rows -- from ONE read of V, through LDS, where the
// unfused path streams V twice more (gnk_basis_gemv_pending, then gnk_vjp_gemv_t; ref:krylow.py:62-64,
// ref:armijo_goldstein.py:56).  A workgroup (4 waves) walks TP-point tiles of one grid row (TP = 128 up to 104
// columns, 64 beyond: the tile's kk columns fit LDS), tiles t = blockIdx.x + i gridDim.x of a fixed grid (the
// reduction decomposition: a function of N, the slab and the width class only); the kk columns of the next DEPTH
// tiles are loaded as 16-B pairs into VGPRs while tile t is computed from LDS:
//   A. wave w, lane = TP / 64 consecutive points: its quarter of the settled columns, s_w = sum V_j hh_j and
//      xs_w = sum V_j c_j;
//   B. wave 0: w = wcol - (((s_0 + s_1) + s_2) + s_3), x = (((xs_0 + xs_1) + xs_2) + xs_3) + w c_k (stored, w
//      written over its column, in LDS too), on owned rows g = -J(x)^T r at the point -> store and LDS;
//   C. thread j < kk: h_j += the tile's sum of V'_j g (V'_k = w): four point chains, combined in a fixed order.
// Block partials: h at partial[blk * kk + j], {sum w^2, max |w|} at spart[2 blk].
constexpr int TW_KMAX = 208;              // widest basis (kk = k + pending) of the kernel
template <int TP, int ROUNDS, int DEPTH, bool PEND, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void k_trial_w(const double* __restrict__ V,
                                                   int64_t ldv, int k,
                                                   const double* __restrict__ cvec, const double* __restrict__ hh,
                                                   double* __restrict__ wcol, const double* __restrict__ r,
                                                   double* __restrict__ x, double* __restrict__ g, Geo geo, Coef c,
                                                   int64_t ntiles, double* __restrict__ partial,
                                                   double* __restrict__ spart) {
  constexpr int LD = TP + 2;                          // LDS column stride (doubles): 16-B aligned, spreads stage C
  constexpr int PPL = TP / 64;                        // points per lane in stages A and B (consecutive)
  constexpr int HALF = TP / 2;                        // 16-B pairs per column
  constexpr int CPR = BLOCK / HALF;                   // columns per load round
  extern __shared__ __attribute__((aligned(16))) double tw[];
  const int kk = PEND ? k + 1 : k;                    // columns entering x and h
  const int ks = k;                                   // settled columns read in stage A (PEND: w separately)
  double* Vt = tw;                                    // [kk][LD]
  double* gl = Vt + size_t(kk) * LD;                  // g of the tile's points
  double* sp = gl + TP;                               // stage-A partials [2][4][TP]: s, then xs
  double* cl = sp + 8 * TP;                           // c[0 .. kk)
  double* hl = cl + kk;                               // hh[0 .. k)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t N = geo.N;
  const int64_t tpr = N / TP;                         // tiles per grid row
  const int64_t GS = gridDim.x;                       // tile stride
  for (int j = tid; j < kk; j += BLOCK) cl[j] = cvec[j];
  if (PEND)
    for (int j = tid; j < k; j += BLOCK) hl[j] = hh[j];
  // this thread's pair of every load round: column CPR rho + tid / HALF, points 2 (tid % HALF) .. + 1
  const int jc0 = tid / HALF, q2 = 2 * (tid % HALF);
  // DEPTH tiles' columns in flight in VGPRs (buffer b: st_b; r_b = wave 0's r of the tile's points (PPL), the
  // rows above / below, and the strip's outer neighbour for lanes 0 / 63)
  d2 st0[ROUNDS], st1[DEPTH == 2 ? ROUNDS : 1];
  double r0[3 * PPL + 1] = {}, r1[3 * PPL + 1] = {};
  auto load = [&](int64_t t, d2* st, double* rr) {
    const int64_t lr = t / tpr, li0 = lr * N + (t % tpr) * TP;
#pragma unroll
    for (int rho = 0; rho < ROUNDS; ++rho) {
      const int j = CPR * rho + jc0;
      if (j < kk) st[rho] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(V + int64_t(j) * ldv + li0 + q2));
    }
    if (wave == 0 && lr >= G && lr < G + geo.nrows) {
      const int64_t i = li0 + PPL * lane;
      if constexpr (PPL == 2) {
        const d2 a = *reinterpret_cast<const d2*>(r + i), b = *reinterpret_cast<const d2*>(r + i - N);
        const d2 cc = *reinterpret_cast<const d2*>(r + i + N);
        rr[0] = a.x; rr[1] = a.y; rr[2] = b.x; rr[3] = b.y; rr[4] = cc.x; rr[5] = cc.y;
      } else {
        rr[0] = r[i];
        rr[1] = r[i - N];
        rr[2] = r[i + N];
      }
      // lane 0: the west neighbour of the tile's first point, lane 63: the east one of its last (0 at the domain edge)
      const int64_t iy0 = (t % tpr) * TP;
      rr[3 * PPL] = lane == 0 ? (iy0 > 0 ? r[li0 - 1] : 0.0) : (lane == 63 ? (iy0 + TP < N ? r[li0 + TP] : 0.0) : 0.0);
    }
  };
  auto stage = [&](const d2* st) {
#pragma unroll
    for (int rho = 0; rho < ROUNDS; ++rho) {
      const int j = CPR * rho + jc0;
      if (j < kk) *reinterpret_cast<d2*>(Vt + j * LD + q2) = st[rho];
    }
  };
  double acc = 0.0, ss = 0.0, mx = 0.0;
  // tile t from LDS (its r in rr); ends with every wave past its LDS reads
  auto tile = [&](int64_t t, const double* rr) {
    const int64_t lr = t / tpr, li0 = lr * N + (t % tpr) * TP;
    const bool owned = lr >= G && lr < G + geo.nrows;          // block-uniform
    const int p0 = PPL * lane;                                 // this lane's first point in the tile
    // A: wave w sums columns [w Q, (w + 1) Q) of the settled ones in column order, per point
    {
      const int Q = (ks + 3) / 4;
      const int j0 = wave * Q, j1 = min(ks, j0 + Q);
      double s[PPL] = {}, xs[PPL] = {};
      for (int j = j0; j < j1; ++j) {
        double v[PPL];
        if constexpr (PPL == 2) {
          const d2 vv = *reinterpret_cast<const d2*>(Vt + j * LD + p0);
          v[0] = vv.x;
          v[1] = vv.y;
        } else {
          v[0] = Vt[j * LD + p0];
        }
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
          if (PEND) s[q] = s[q] + v[q] * hl[j];
          xs[q] = xs[q] + v[q] * cl[j];
        }
      }
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        sp[wave * TP + p0 + q] = s[q];
        sp[(4 + wave) * TP + p0 + q] = xs[q];
      }
    }
    __syncthreads();
    // B: wave 0 combines, materialises w, stores x, forms g on owned rows
    if (wave == 0) {
      double xv[PPL];
#pragma unroll
      for (int q = 0; q < PPL; ++q) {
        const int p = p0 + q;
        double xs = ((sp[4 * TP + p] + sp[5 * TP + p]) + sp[6 * TP + p]) + sp[7 * TP + p];
        if (PEND) {
          const double sw = ((sp[p] + sp[TP + p]) + sp[2 * TP + p]) + sp[3 * TP + p];
          const double wv = Vt[k * LD + p] - sw;
          Vt[k * LD + p] = wv;
          st_nt(wcol + li0 + p, wv);
          xs = xs + wv * cl[k];
          if (owned) {
            ss += wv * wv;
            mx = nan_max(mx, fabs(wv));
          }
        }
        xv[q] = xs;
      }
      if constexpr (PPL == 2) st_nt(x + li0 + p0, d2{xv[0], xv[1]});
      else st_nt(x + li0 + p0, xv[0]);
      if (owned) {
        const int64_t iy = (t % tpr) * TP + p0;
        const double re_ = rr[3 * PPL];
        double gv[PPL];
        if constexpr (PPL == 2) {
          // points 2l, 2l + 1: rc = (rr[0], rr[1]), north (rr[2], rr[3]), south (rr[4], rr[5])
          double rw = lane_prev(rr[1]), re = lane_next(rr[0]);
          if (lane == 0) rw = re_;
          if (lane == 63) re = re_;
          gv[0] = -vjp_pt(c, jdiag(c, xv[0]), rr[2], rw, iy > 0, rr[0], rr[1], true, rr[4]);
          gv[1] = -vjp_pt(c, jdiag(c, xv[1]), rr[3], rr[0], true, rr[1], re, iy + 2 < N, rr[5]);
          st_nt(g + li0 + p0, d2{gv[0], gv[1]});
        } else {
          double rw = lane_prev(rr[0]), re = lane_next(rr[0]);
          if (lane == 0) rw = re_;
          if (lane == 63) re = re_;
          gv[0] = -vjp_pt(c, jdiag(c, xv[0]), rr[1], rw, iy > 0, rr[0], re, iy + 1 < N, rr[2]);
          st_nt(g + li0 + p0, gv[0]);
        }
#pragma unroll
        for (int q = 0; q < PPL; ++q) gl[p0 + q] = gv[q];
      }
    }
    __syncthreads();
    // C: thread j accumulates V'_j . g over the tile's points: four chains (points p = 4i + m, i ascending),
    // ((a_0 + a_1) + a_2) + a_3 added to the running sum -- short dependency chains, a fixed order
    if (owned && tid < kk) {
      const double* col = Vt + tid * LD;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll 2
      for (int p = 0; p < TP; p += 4) {
        a0 = a0 + col[p] * gl[p];
        a1 = a1 + col[p + 1] * gl[p + 1];
        a2 = a2 + col[p + 2] * gl[p + 2];
        a3 = a3 + col[p + 3] * gl[p + 3];
      }
      acc = acc + (((a0 + a1) + a2) + a3);
    }
    __syncthreads();
  };
  int64_t t = blockIdx.x;
  if (t < ntiles) {
    load(t, st0, r0);
    stage(st0);
  }
  if (DEPTH == 2 && t + GS < ntiles) load(t + GS, st1, r1);
  __syncthreads();
  while (t < ntiles) {
    // tile t in LDS, its r in r0; st0 free (staged); DEPTH 2: st1 holds tile t + GS
    {
      double cur[3 * PPL + 1];
#pragma unroll
      for (int q = 0; q < 3 * PPL + 1; ++q) cur[q] = r0[q];
      const int64_t tl = t + DEPTH * GS;                       // the next free buffer's tile
      if (tl < ntiles) load(tl, st0, r0);
      tile(t, cur);
      if (t + GS < ntiles) stage(DEPTH == 2 ? st1 : st0);
      __syncthreads();
      t += GS;
    }
    if (DEPTH == 1 || t >= ntiles) continue;
    // tile t in LDS, its r in r1; st1 free; st0 holds tile t + GS
    {
      double cur[3 * PPL + 1];
#pragma unroll
      for (int q = 0; q < 3 * PPL + 1; ++q) cur[q] = r1[q];
      if (t + 2 * GS < ntiles) load(t + 2 * GS, st1, r1);
      tile(t, cur);
      if (t + GS < ntiles) stage(st0);
      __syncthreads();
      t += GS;
    }
  }
  if (tid < kk) partial[size_t(blockIdx.x) * kk + tid] = acc;
  if (PEND) block_sum_max_store(wave == 0 ? ss : 0.0, wave == 0 ? mx : 0.0, spart);
}

// g -= V[:, :k] @ h ; partial {sum g^2, max|g|}
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_cgs(const double* __restrict__ V, int64_t ldv, int k,
                                               const double* __restrict__ h, double* __restrict__ g, Geo geo,
                                               int64_t lr0, int64_t nlr, double* __restrict__ partial) {
  __shared__ double sh[BLOCK / 64][2];
  double ss = 0.0, mx = 0.0;
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    d2 s = {0.0, 0.0};
    for (int j = 0; j < k; ++j) {
      const d2 vv = *reinterpret_cast<const d2*>(V + j * ldv + li);
      const double hj = h[j];
      s.x = s.x + vv.x * hj;
      s.y = s.y + vv.y * hj;
    }
    d2 gg = *reinterpret_cast<const d2*>(g + li);
    gg.x = gg.x - s.x;
    gg.y = gg.y - s.y;
    *reinterpret_cast<d2*>(g + li) = gg;
    ss += gg.x * gg.x;
    ss += gg.y * gg.y;
    mx = nan_max(mx, fabs(gg.x));
    mx = nan_max(mx, fabs(gg.y));
  } else {
    for (int q = 0; q < VEC && iy + q < N; ++q) {
      double s = 0.0;
      for (int j = 0; j < k; ++j) s = s + V[j * ldv + li + q] * h[j];
      const double gi = g[li + q] - s;
      g[li + q] = gi;
      ss += gi * gi;
      mx = nan_max(mx, fabs(gi));
    }
  }
  ROW_LOOP_END
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  ss = wave_sum(ss);
  mx = wave_max(mx);
  if (lane == 0) { sh[wave][0] = ss; sh[wave][1] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = sh[0][0], b = sh[0][1];
    for (int w = 1; w < BLOCK / 64; ++w) { a += sh[w][0]; b = nan_max(b, sh[w][1]); }
    const size_t blk = blockIdx.y * gridDim.x + blockIdx.x;
    partial[2 * blk] = a;
    partial[2 * blk + 1] = b;
  }
}

// {sum x^2, max |x|}
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_stats(const double* __restrict__ x, Geo geo, int64_t lr0, int64_t nlr,
                                                 double* __restrict__ partial) {
  __shared__ double sh[BLOCK / 64][3];
  double ss = 0.0, sc = 0.0, mx = 0.0;
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {                     // one 16-B pair, the loop's order point by point
    const d2 xv = *reinterpret_cast<const d2*>(x + li);
    comp_dot(ss, sc, xv.x, xv.x);
    mx = nan_max(mx, fabs(xv.x));
    comp_dot(ss, sc, xv.y, xv.y);
    mx = nan_max(mx, fabs(xv.y));
  } else {
    for (int q = 0; q < VEC && iy + q < N; ++q) {
      const double xi = x[li + q];
      comp_dot(ss, sc, xi, xi);
      mx = nan_max(mx, fabs(xi));
    }
  }
  ROW_LOOP_END
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  wave_sum2(ss, sc);
  mx = wave_max(mx);
  if (lane == 0) { sh[wave][0] = ss; sh[wave][1] = sc; sh[wave][2] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = sh[0][0], ac = sh[0][1], b = sh[0][2];
    for (int w = 1; w < BLOCK / 64; ++w) { comp_merge(a, ac, sh[w][0], sh[w][1]); b = nan_max(b, sh[w][2]); }
    const size_t blk = blockIdx.y * gridDim.x + blockIdx.x;
    partial[3 * blk] = a;                           // {sum x^2 as s + c, max |x|}
    partial[3 * blk + 1] = ac;
    partial[3 * blk + 2] = b;
  }
}

template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_div(const double* __restrict__ src, double denom, double* __restrict__ dst,
                                               Geo geo, int64_t lr0, int64_t nlr) {
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    const d2 sv = *reinterpret_cast<const d2*>(src + li);
    *reinterpret_cast<d2*>(dst + li) = d2{sv.x / denom, sv.y / denom};
  } else {
    for (int q = 0; q < VEC && iy + q < N; ++q) dst[li + q] = src[li + q] / denom;
  }
  ROW_LOOP_END
}

// v = g / denom on the whole slab (g's ghost rows already exchanged, so each rank's
// ghost copy equals its neighbour's owned value bit for bit) and, on owned rows,
// partial sum of (J(u) g)^2 from the same loads; the host divides by denom^2 to get
// ||J v_new||^2, the appended column's scale in the next least-squares preconditioner
// (not a parity quantity: one division per point instead of five).  v must not alias g.
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_div_jnorm(const double* __restrict__ u, const double* __restrict__ g,
                                                     double denom, double* __restrict__ v, Geo geo, Coef c,
                                                     int64_t lr0, int64_t nlr, double* __restrict__ partial) {
  __shared__ double sh[BLOCK / 64];
  const int lane = threadIdx.x & 63;
  double acc[1] = {0.0};
  ROW_LOOP_BEGIN(VEC)
  const bool owned = lr >= G && lr < G + geo.nrows;   // block-uniform
  if (!owned) {
    for (int q = 0; q < VEC && iy + q < N; ++q) v[li + q] = g[li + q] / denom;
    continue;
  }
  if (VEC == 2 && iy + 1 < N) {
    const d2 uc = *reinterpret_cast<const d2*>(u + li);
    const d2 gc = *reinterpret_cast<const d2*>(g + li);
    const d2 gn = *reinterpret_cast<const d2*>(g + li - N);
    const d2 gs = *reinterpret_cast<const d2*>(g + li + N);
    const bool hw = iy > 0, he = iy + 2 < N;
    double gw = __shfl_up(gc.y, 1);
    double ge = __shfl_down(gc.x, 1);
    if (lane == 0) gw = hw ? g[li - 1] : 0.0;
    if (lane == 63 || iy + 2 >= N) ge = he ? g[li + 2] : 0.0;
    *reinterpret_cast<d2*>(v + li) = d2{gc.x / denom, gc.y / denom};
    const double j0 = jvp_pt(c, jdiag(c, uc.x), gn.x, gw, hw, gc.x, gc.y, true, gs.x);
    const double j1 = jvp_pt(c, jdiag(c, uc.y), gn.y, gc.x, true, gc.y, ge, he, gs.y);
    acc[0] += j0 * j0;
    acc[0] += j1 * j1;
  } else {
    for (int q = 0; q < VEC; ++q) {
      const int64_t i = li + q;
      const int64_t y = iy + q;
      if (y >= N) break;
      const bool hw = y > 0, he = y < N - 1;
      v[i] = g[i] / denom;
      const double gw = hw ? g[i - 1] : 0.0, ge = he ? g[i + 1] : 0.0;
      const double jg = jvp_pt(c, jdiag(c, u[i]), g[i - N], gw, hw, g[i], ge, he, g[i + N]);
      acc[0] += jg * jg;
    }
  }
  ROW_LOOP_END
  block_sum_store<1>(acc, 1, partial + (blockIdx.y * gridDim.x + blockIdx.x), sh);
}

// out = x + (alpha * d): the two roundings of NumPy's `x + step_length * descent_direction`
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_axpy(const double* __restrict__ x, double alpha, const double* __restrict__ d,
                                                double* __restrict__ out, Geo geo, int64_t lr0, int64_t nlr) {
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    const d2 dv = *reinterpret_cast<const d2*>(d + li), xv = *reinterpret_cast<const d2*>(x + li);
    const double t0 = alpha * dv.x, t1 = alpha * dv.y;
    *reinterpret_cast<d2*>(out + li) = d2{xv.x + t0, xv.y + t1};
  } else {
    for (int q = 0; q < VEC && iy + q < N; ++q) {
      const double td = alpha * d[li + q];
      out[li + q] = x[li + q] + td;
    }
  }
  ROW_LOOP_END
}

// ---------------------------------------------------------------- CG kernels
// d = diag of (L + ALPHA D_x + LAMBDA diag e^u), constant during a CG solve
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_jdiag(const double* __restrict__ u, double* __restrict__ d, Geo geo,
                                                 Coef c, int64_t lr0, int64_t nlr) {
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    const d2 uv = *reinterpret_cast<const d2*>(u + li);
    *reinterpret_cast<d2*>(d + li) = d2{jdiag(c, uv.x), jdiag(c, uv.y)};
  } else {
    for (int q = 0; q < VEC && iy + q < N; ++q) d[li + q] = jdiag(c, u[li + q]);
  }
  ROW_LOOP_END
}

// (J p)_j for a point j of row gj (outside the domain -> 0)
__device__ __forceinline__ double tj(const Coef& c, const double* __restrict__ d, const double* __restrict__ p,
                                     int64_t j, int64_t gj, int64_t jy, int64_t N) {
  if (gj < 0 || gj >= N) return 0.0;
  const bool hw = jy > 0, he = jy < N - 1;
  const double pw = hw ? p[j - 1] : 0.0, pe = he ? p[j + 1] : 0.0;
  return jvp_pt(c, d[j], p[j - N], pw, hw, p[j], pe, he, p[j + N]);
}

// q = J^T (J p), 13-point fused; identical arithmetic to t = J p followed by q = J^T t
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_cg_matvec(const double* __restrict__ d, const double* __restrict__ p,
                                                     double* __restrict__ q, Geo geo, Coef c, int64_t lr0,
                                                     int64_t nlr, double* __restrict__ partial) {
  __shared__ double sh[BLOCK / 64 * 2];
  double acc[1] = {0.0}, accc[1] = {0.0};
  ROW_LOOP_BEGIN(VEC)
  const int64_t gr = geo.row0 + (lr - G);
#pragma unroll
  for (int qq = 0; qq < VEC; ++qq) {
    const int64_t i = li + qq;
    const int64_t yy = iy + qq;
    if (yy >= N) break;
    const bool hw = yy > 0, he = yy < N - 1;
    const double tn = tj(c, d, p, i - N, gr - 1, yy, N);
    const double tw = hw ? tj(c, d, p, i - 1, gr, yy - 1, N) : 0.0;
    const double tc = tj(c, d, p, i, gr, yy, N);
    const double te = he ? tj(c, d, p, i + 1, gr, yy + 1, N) : 0.0;
    const double ts = tj(c, d, p, i + N, gr + 1, yy, N);
    const double qi = vjp_pt(c, d[i], tn, tw, hw, tc, te, he, ts);
    q[i] = qi;
    comp_dot(acc[0], accc[0], p[i], qi);
  }
  ROW_LOOP_END
  block_sum2_store<1>(acc, accc, 1, partial + 2 * (blockIdx.y * gridDim.x + blockIdx.x), sh);
}

// q = J^T (J p) by row marching, and the partial p.q.  One wave walks a 128-point strip (two points
// per lane) down a range of rows, four strips per block.  t = J p of rows x-1, x, x+1 stays in
// registers, so every p and d value is loaded once per range (+2 warm-up rows) instead of up to 13
// times.  The in-row neighbours of p and t come from the adjacent lanes.  At the strip edges:
//   * lanes 0 and 63 load one extra 16-B pair of p and d per row;
//   * they evaluate the one t point outside the strip.
// Each point is computed as in k_cg_matvec (jvp_pt then vjp_pt, same operands, same order), so q
// is bit-identical; only the p.q partial sums are grouped differently.  Requires N even (16-B pairs).
//
// FUSED: the CG direction update of the same iteration rides on the loads (scipy iterative.py:
// 401-415 order kept): p = first ? z : p_in * beta + z is formed as each row of z / p_in streams in
// and stored to p (never p_in: neighbouring ranges read the overlap rows); the ranges at the slab
// ends also store the ghost rows, so with z's halo exchanged every rank holds its neighbours' p
// bit for bit.  x (optional) takes the previous iteration's x += xalpha * p_in on owned rows at the
// same point (one iteration late; the caller applies the last one).
constexpr int CGM_SW = 128;

template <bool FUSED>
__global__ __launch_bounds__(BLOCK) void k_cg_matvec_m(const double* __restrict__ d, const double* __restrict__ pin,
                                                       double* __restrict__ q, Geo geo, Coef c, int64_t rpr,
                                                       double* __restrict__ partial, const double* __restrict__ z,
                                                       double* __restrict__ p, double beta, int first,
                                                       double* __restrict__ x, double xalpha,
                                                       const double* __restrict__ cst) {
  __shared__ double sh[BLOCK / 64 * 2];
  if (cst) {                       // device CG state (gnk_cg_scalars): beta = cst[0], lagged alpha = cst[1]
    beta = cst[0];
    xalpha = cst[1];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t N = geo.N;
  const int nbc = int((N + 4 * CGM_SW - 1) / (4 * CGM_SW));
  const int nwg = gridDim.x, b = blockIdx.x;
  // XCD-aware: consecutive tiles of one XCD (blockIdx % 8) are neighbouring strips of a row range
  const int idx = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
  const int64_t x0 = int64_t(idx / nbc) * rpr;            // owned-row index range [x0, x1)
  const int64_t x1 = min(geo.nrows, x0 + rpr);
  const int64_t col0 = int64_t(idx % nbc) * (4 * CGM_SW) + wave * CGM_SW;
  const int64_t y0 = col0 + 2 * lane;                     // this lane's points y0, y0 + 1
  const bool valid = y0 < N;
  const bool hw0 = y0 > 0, he1 = y0 + 2 < N;
  // edge pairs: lane 0 -> columns col0-2, col0-1; lane 63 -> col0+128, col0+129
  const bool ex = (lane == 0 && col0 > 0) || (lane == 63 && col0 + CGM_SW < N);
  const int64_t exo = lane == 0 ? -2 : 2;
  double acc[1] = {0.0}, accc[1] = {0.0};
  auto ld = [&](const double* base, int64_t xr) -> d2 {   // xr: owned-row index (may be -2 .. nrows+1)
    return valid ? *reinterpret_cast<const d2*>(base + (G + xr) * N + y0) : d2{0.0, 0.0};
  };
  auto ldx = [&](const double* base, int64_t xr) -> d2 {
    return ex ? *reinterpret_cast<const d2*>(base + (G + xr) * N + y0 + exo) : d2{0.0, 0.0};
  };
  auto pnew = [&](d2 zz, d2 pp) -> d2 {                  // k_cg_p's arithmetic
    return first ? zz : d2{pp.x * beta + zz.x, pp.y * beta + zz.y};
  };
  // row xr of the direction: loaded (plain) or formed and stored (FUSED, + the lagged x update)
  auto ldp = [&](int64_t xr) -> d2 {
    if (!FUSED) return ld(pin, xr);
    const d2 pi = ld(pin, xr);
    const d2 pv = pnew(ld(z, xr), pi);
    const bool own = xr >= x0 && xr < x1;
    const bool ghost = (x0 == 0 && xr < 0) || (x1 == geo.nrows && xr >= geo.nrows);
    // non-temporal stores (p, x, q are re-read only by the next kernels, after other streams): -0.9 % per CG
    // iteration at 8192^2, bit-identical (profiles/round6/cg_nt_ab.jsonl)
    if (valid && (own || ghost)) st_nt(p + (G + xr) * N + y0, pv);
    if (x && valid && own) {
      double* xp = x + (G + xr) * N + y0;
      const d2 xv = *reinterpret_cast<const d2*>(xp);
      st_nt(xp, d2{xv.x + xalpha * pi.x, xv.y + xalpha * pi.y});
    }
    return pv;
  };
  auto ldpx = [&](int64_t xr) -> d2 {
    if (!FUSED) return ldx(pin, xr);
    return ex ? pnew(ldx(z, xr), ldx(pin, xr)) : d2{0.0, 0.0};
  };
  // t = J p at this lane's two points of row x (0 outside the domain)
  auto trow = [&](int64_t xr, d2 pn, d2 pc, d2 ps, d2 xc, d2 dc) -> d2 {
    double pw = lane_prev(pc.y);
    double pe = lane_next(pc.x);
    if (lane == 0) pw = xc.y;
    if (lane == 63) pe = xc.x;
    const int64_t gx = geo.row0 + xr;
    if (gx < 0 || gx >= N || !valid) return d2{0.0, 0.0};
    d2 t;
    t.x = jvp_pt(c, dc.x, pn.x, pw, hw0, pc.x, pc.y, true, ps.x);
    t.y = jvp_pt(c, dc.y, pn.y, pc.x, true, pc.y, pe, he1, ps.y);
    return t;
  };
  if (x0 < x1) {
    // rows x-1 .. x+2 of p (and edge pairs), rows x, x+1 of d, t rows x-1, x
    d2 pA = ldp(x0 - 2), pB = ldp(x0 - 1), pC = ldp(x0), pD = ldp(x0 + 1), pE = ldp(x0 + 2);
    d2 xA = ldpx(x0 - 1), xB = ldpx(x0), xC = ldpx(x0 + 1), xD = ldpx(x0 + 2);
    d2 dA = ld(d, x0 - 1), dB = ld(d, x0), dC = ld(d, x0 + 1);
    d2 eB = ldx(d, x0), eC = ldx(d, x0 + 1);
    d2 tn = trow(x0 - 1, pA, pB, pC, xA, dA);
    d2 tc = trow(x0, pB, pC, pD, xB, dB);
    // loop invariants: pB, pC, pD, pE = p rows x-1 .. x+2; xA, xB, xC = edge pairs x-1 .. x+1,
    // xD = x+2; dB, dC = d rows x, x+1; eB, eC = their edge pairs
    for (int64_t xs = x0; xs < x1; ++xs) {
      // prefetch row x+3 of p and row x+2 of d for the next step
      const bool more = xs + 1 < x1;
      const d2 pF = more ? ldp(xs + 3) : d2{0.0, 0.0};
      const d2 xE = more ? ldpx(xs + 3) : d2{0.0, 0.0};
      const d2 dD = more ? ld(d, xs + 2) : d2{0.0, 0.0};
      const d2 eD = more ? ldx(d, xs + 2) : d2{0.0, 0.0};
      const d2 ts = trow(xs + 1, pC, pD, pE, xC, dC);
      // the t point just outside the strip, row x (lane 0: col0-1; lane 63: col0+128)
      const bool l0 = lane == 0;
      const double te = jvp_pt(c, l0 ? eB.y : eB.x, l0 ? xA.y : xA.x, l0 ? xB.x : pC.y, l0 ? col0 - 1 > 0 : true,
                               l0 ? xB.y : xB.x, l0 ? pC.x : xB.y, l0 ? true : col0 + CGM_SW < N - 1,
                               l0 ? xC.y : xC.x);
      double tw = lane_prev(tc.y);
      double tE = lane_next(tc.x);
      if (lane == 0) tw = te;
      if (lane == 63) tE = te;
      if (valid) {
        d2 qo;
        qo.x = vjp_pt(c, dB.x, tn.x, tw, hw0, tc.x, tc.y, true, ts.x);
        qo.y = vjp_pt(c, dB.y, tn.y, tc.x, true, tc.y, tE, he1, ts.y);
        st_nt(q + (G + xs) * N + y0, qo);
        comp_dot(acc[0], accc[0], pC.x, qo.x);
        comp_dot(acc[0], accc[0], pC.y, qo.y);
      }
      tn = tc;
      tc = ts;
      pB = pC; pC = pD; pD = pE; pE = pF;
      xA = xB; xB = xC; xC = xD; xD = xE;
      dB = dC; dC = dD;
      eB = eC; eC = eD;
    }
  }
  block_sum2_store<1>(acc, accc, 1, partial + 2 * blockIdx.x, sh);
}

template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_cg_xr(double alpha, const double* __restrict__ p,
                                                 const double* __restrict__ q, double* __restrict__ x,
                                                 double* __restrict__ r, const double* __restrict__ dinv,
                                                 double* __restrict__ z, Geo geo, int64_t lr0, int64_t nlr,
                                                 double* __restrict__ partial, const double* __restrict__ cst) {
  __shared__ double sh[(BLOCK / 64) * 2 * 2];
  if (cst) alpha = cst[2];         // device CG state (gnk_cg_scalars)
  double acc[2] = {0.0, 0.0}, accc[2] = {0.0, 0.0};
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    // the two points as 16-B pairs (the loop below's arithmetic and accumulation order, point by point)
    if (x) {                                           // NULL x: done by the fused matvec (lagged)
      const d2 pv = *reinterpret_cast<const d2*>(p + li);
      d2 xv = *reinterpret_cast<const d2*>(x + li);
      xv.x = xv.x + alpha * pv.x;
      xv.y = xv.y + alpha * pv.y;
      *reinterpret_cast<d2*>(x + li) = xv;
    }
    const d2 qv = *reinterpret_cast<const d2*>(q + li);
    d2 rv = *reinterpret_cast<const d2*>(r + li);
    rv.x = rv.x - alpha * qv.x;
    rv.y = rv.y - alpha * qv.y;
    *reinterpret_cast<d2*>(r + li) = rv;
    d2 zv = rv;
    if (dinv) {
      const d2 dv = *reinterpret_cast<const d2*>(dinv + li);
      zv.x = 0.0 + dv.x * rv.x;
      zv.y = 0.0 + dv.y * rv.y;
      *reinterpret_cast<d2*>(z + li) = zv;
    }
    comp_dot(acc[0], accc[0], rv.x, rv.x);
    comp_dot(acc[1], accc[1], rv.x, zv.x);
    comp_dot(acc[0], accc[0], rv.y, rv.y);
    comp_dot(acc[1], accc[1], rv.y, zv.y);
  } else {
    for (int qq = 0; qq < VEC && iy + qq < N; ++qq) {
      const int64_t i = li + qq;
      if (x) x[i] = x[i] + alpha * p[i];
      const double ri = r[i] - alpha * q[i];
      r[i] = ri;
      const double zi = dinv ? 0.0 + dinv[i] * ri : ri;
      if (dinv) z[i] = zi;
      comp_dot(acc[0], accc[0], ri, ri);
      comp_dot(acc[1], accc[1], ri, zi);
    }
  }
  ROW_LOOP_END
  block_sum2_store<2>(acc, accc, 2, partial + 4 * (blockIdx.y * gridDim.x + blockIdx.x), sh);
}

// Single-reduction CG iteration (Chronopoulos-Gear; the build's non-parity option) on
// owned rows: p = u + beta p, s = w + beta s (first: p = u, s = w); x += alpha p; r -= alpha s;
// u = M r (dinv NULL: u = r); partials {r . u, r . r}.  With w = A^T A u from the normal matvec and
// its u . w, one host read per iteration carries all three scalars.
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_cg_sr(double alpha, double beta, int first, const double* __restrict__ w,
                                                 double* __restrict__ p, double* __restrict__ sv,
                                                 double* __restrict__ x, double* __restrict__ r,
                                                 const double* __restrict__ dinv, double* __restrict__ u, Geo geo,
                                                 int64_t lr0, int64_t nlr, double* __restrict__ partial) {
  __shared__ double sh[(BLOCK / 64) * 2];
  double acc[2] = {0.0, 0.0};
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    // 16-B pairs; the loop's arithmetic and accumulation order point by point
    const d2 uv = *reinterpret_cast<const d2*>(u + li), wv = *reinterpret_cast<const d2*>(w + li);
    d2 pv = uv, sv2 = wv;
    if (!first) {
      const d2 po = *reinterpret_cast<const d2*>(p + li), so = *reinterpret_cast<const d2*>(sv + li);
      pv = d2{uv.x + beta * po.x, uv.y + beta * po.y};
      sv2 = d2{wv.x + beta * so.x, wv.y + beta * so.y};
    }
    *reinterpret_cast<d2*>(p + li) = pv;
    *reinterpret_cast<d2*>(sv + li) = sv2;
    d2 xv = *reinterpret_cast<const d2*>(x + li);
    xv.x = xv.x + alpha * pv.x;
    xv.y = xv.y + alpha * pv.y;
    *reinterpret_cast<d2*>(x + li) = xv;
    d2 rv = *reinterpret_cast<const d2*>(r + li);
    rv.x = rv.x - alpha * sv2.x;
    rv.y = rv.y - alpha * sv2.y;
    *reinterpret_cast<d2*>(r + li) = rv;
    d2 un = rv;
    if (dinv) {
      const d2 dv = *reinterpret_cast<const d2*>(dinv + li);
      un = d2{0.0 + dv.x * rv.x, 0.0 + dv.y * rv.y};
    }
    *reinterpret_cast<d2*>(u + li) = un;
    acc[0] += rv.x * un.x;
    acc[1] += rv.x * rv.x;
    acc[0] += rv.y * un.y;
    acc[1] += rv.y * rv.y;
  } else {
    for (int qq = 0; qq < VEC && iy + qq < N; ++qq) {
      const int64_t i = li + qq;
      const double pi = first ? u[i] : u[i] + beta * p[i];
      const double si = first ? w[i] : w[i] + beta * sv[i];
      p[i] = pi;
      sv[i] = si;
      x[i] = x[i] + alpha * pi;
      const double ri = r[i] - alpha * si;
      r[i] = ri;
      const double ui = dinv ? 0.0 + dinv[i] * ri : ri;
      u[i] = ui;
      acc[0] += ri * ui;
      acc[1] += ri * ri;
    }
  }
  ROW_LOOP_END
  block_sum_store<2>(acc, 2, partial + 2 * (blockIdx.y * gridDim.x + blockIdx.x), sh);
}

template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_cg_p(double beta, int first, const double* __restrict__ z,
                                                double* __restrict__ p, Geo geo, int64_t lr0, int64_t nlr) {
  ROW_LOOP_BEGIN(VEC)
  if (VEC == 2 && iy + 1 < N) {
    const d2 zv = *reinterpret_cast<const d2*>(z + li);
    if (first) {
      *reinterpret_cast<d2*>(p + li) = zv;
    } else {
      const d2 pv = *reinterpret_cast<const d2*>(p + li);
      *reinterpret_cast<d2*>(p + li) = d2{pv.x * beta + zv.x, pv.y * beta + zv.y};
    }
  } else {
    for (int qq = 0; qq < VEC && iy + qq < N; ++qq) {
      const int64_t i = li + qq;
      p[i] = first ? z[i] : p[i] * beta + z[i];
    }
  }
  ROW_LOOP_END
}

// Device-side scalar recurrence of the fused scipy-cg iteration (DeviceCG._cg_fused_dev): merges the ranks'
// compensated (s, c) pairs exactly as slab.Comm.merge_pairs does on the host (TwoSum in rank order, the
// errors and the c accumulated beside, one rounding at the end; one rank: s + c) and forms the step
// coefficients of scipy iterative.py:305-422 where the host formed them: the same IEEE operations, so the
// kernels that read them compute the same bits, and no host read sits between two kernels.
// state: [0] beta = rho / rho_prev  [1] the lagged alpha of the x update  [2] alpha = rho / (p . q)
//        [3] rho = r . z  [4] rho_prev  [5] r . r  [6] p . q
// stage 0 (the alpha = 0 update that forms z = M r; parts: rank x [s, c](r.r), [s, c](r.z)): r.r, rho
// stage 1 (after the normal matvec; parts: rank x [s, c](p.q)):  alpha = rho / p.q
// stage 2 (after the r, z update; parts as stage 0): r.r; rho_prev = rho, rho = r.z, beta = rho / rho_prev,
//         the lagged alpha = alpha
__device__ double merge_pair(const double* __restrict__ parts, int world, int stride, int q) {
  double S = parts[2 * q], C = parts[2 * q + 1];
  for (int w = 1; w < world; ++w) {
    const double sp = parts[w * stride + 2 * q], cp = parts[w * stride + 2 * q + 1];
    const double x = S + sp;
    const double z = x - S;
    const double err = (S - (x - z)) + (sp - z);
    S = x;
    C = C + (err + cp);
  }
  return S + C;
}

__global__ __launch_bounds__(64) void k_cg_scalars(const double* __restrict__ parts, int world, int stage,
                                                   double* __restrict__ st) {
  if (threadIdx.x != 0) return;
  if (stage == 1) {
    const double pq = merge_pair(parts, world, 2, 0);
    st[6] = pq;
    st[2] = st[3] / pq;
    return;
  }
  const double rr = merge_pair(parts, world, 4, 0), rz = merge_pair(parts, world, 4, 1);
  st[5] = rr;
  if (stage == 0) {
    st[0] = 0.0;
    st[1] = 0.0;
    st[2] = 0.0;
    st[3] = rz;
    st[4] = 0.0;
    return;
  }
  st[4] = st[3];
  st[3] = rz;
  st[0] = rz / st[4];
  st[1] = st[2];
}

// ---------------------------------------------------------------- deterministic partial reduction
// sum of all-gathered per-rank partials in the fixed pairwise order of the host (slab.tree_sum) and of
// gnk_set_segments' segment fold: the ranks' values are merged like a binary counter (a new value of
// size 1 merges with the top of the stack while their sizes match, each merge (left) + (right)), then the
// stack folds right to left -- equal to the bottom-up pairwise order v[i] += v[i + w], w = 1, 2, 4, ..
// One launch instead of world - 1 elementwise adds.
__global__ __launch_bounds__(BLOCK) void k_rank_sum(const double* __restrict__ parts, int world, int64_t n,
                                                    double* __restrict__ out) {
  if (world <= 8) {
    // one node: slab.tree_sum's bottom-up pairwise order (v[i] += v[i + w], w = 1, 2, 4), which the binary
    // counter below reproduces, with the values in registers (the counter's stack lives in scratch memory)
    for (int64_t j = int64_t(blockIdx.x) * BLOCK + threadIdx.x; j < n; j += int64_t(gridDim.x) * BLOCK) {
      double v[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) v[p] = p < world ? parts[int64_t(p) * n + j] : 0.0;
#pragma unroll
      for (int w = 1; w < 8; w *= 2)
#pragma unroll
        for (int i = 0; i + w < 8; i += 2 * w)
          if (i + w < world) v[i] = v[i] + v[i + w];
      out[j] = v[0];
    }
    return;
  }
  for (int64_t j = int64_t(blockIdx.x) * BLOCK + threadIdx.x; j < n; j += int64_t(gridDim.x) * BLOCK) {
    double sv[32];
    int sz[32];
    int top = 0;
    for (int p = 0; p < world; ++p) {
      double v = parts[int64_t(p) * n + j];
      int z = 1;
      while (top > 0 && sz[top - 1] == z) {
        v = sv[top - 1] + v;
        z *= 2;
        --top;
      }
      sv[top] = v;
      sz[top] = z;
      ++top;
    }
    double s = sv[--top];
    while (top > 0) s = sv[--top] + s;
    out[j] = s;
  }
}

// Wave-per-output deterministic reduction over a fixed partition of the partials.
// Output j reads partial[base(j) + b * sb] for b in [split * span, min(nblk, (split+1) * span)),
// base(j) = (j / cw) * cs + (j % cw).  Lane l folds b = l, l + 64, ... with 8 independent
// (clamped, branch-free) loads in flight, then a fixed xor-tree.  out[j * nsplit + split].
// segblk > 0 (segment reductions, gnk_set_segments): the blocks come in segments of segblk and no
// split crosses a segment -- split q covers blocks seg * segblk + sub * span .. of segment seg = q / nsps,
// sub = q % nsps (nsps = ceil(segblk / span) splits per segment).
__device__ __forceinline__ void seg_split_range(int split, int span, int nblk, int segblk, int& b0, int& b1) {
  if (segblk > 0) {
    const int nsps = (segblk + span - 1) / span, sg = split / nsps, sub = split % nsps;
    b0 = sg * segblk + sub * span;
    b1 = min(b0 + span, (sg + 1) * segblk);
  } else {
    b0 = split * span;
    b1 = min(nblk, b0 + span);
  }
}

// one wave's deterministic sum (or NaN-propagating max of |x| >= 0) of blocks [b0, b1) of one output: lane-strided
// partial sums (8 loads in flight), then the xor-shuffle tree; shared by every reduction kernel below so that
// a fused form gives the same bits as the separate launches
__device__ __forceinline__ double wave_reduce_range(const double* __restrict__ src, int b0, int b1, int64_t sb, bool mx) {
  const int lane = threadIdx.x & 63;
  double s = mx ? -1.0 : 0.0;    // identity (max is taken over |x| >= 0)
  for (int b = b0 + lane; b < b1; b += 64 * 8) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = src[int64_t(min(b + 64 * q, b1 - 1)) * sb];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (b + 64 * q < b1) s = mx ? nan_max(s, v[q]) : s + v[q];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double t = __shfl_xor(s, o);
    s = mx ? nan_max(s, t) : s + t;
  }
  return (mx && s < 0.0) ? 0.0 : s;
}

__global__ __launch_bounds__(64) void k_wave_reduce(const double* __restrict__ partial, int nblk, int span, int64_t sb,
                                                    int cw, int64_t cs, const int* __restrict__ is_max,
                                                    double* __restrict__ out, int segblk = 0) {
  const int j = blockIdx.x, split = blockIdx.y, nsplit = gridDim.y, lane = threadIdx.x;
  const bool mx = is_max ? is_max[j] != 0 : false;
  const double* src = partial + int64_t(j / cw) * cs + (j % cw);
  int b0, b1;
  seg_split_range(split, span, nblk, segblk, b0, b1);
  const double s = wave_reduce_range(src, b0, b1, sb, mx);
  if (lane == 0) out[int64_t(j) * nsplit + split] = s;
}

// One reduction of the launch-fused forms below: output j < len reads partial[(j / cw) * cs + (j % cw) + b * sb]
// over nblk blocks (per segment: segblk blocks).
struct RedDesc {
  const double* partial;
  int nblk;
  int64_t sb;
  int cw;
  int64_t cs;
  const int* is_max;
  double* out;
  int len;
};

// wreduce of up to two reductions in one launch (each at most 4096 blocks: one split): output j of the
// concatenated range [d0 outputs | d1 outputs]; the arithmetic of k_wave_reduce
__global__ __launch_bounds__(64) void k_wave_reduce_n(RedDesc d0, RedDesc d1) {
  const int jj = blockIdx.x;
  const RedDesc& d = jj < d0.len ? d0 : d1;
  const int j = jj < d0.len ? jj : jj - d0.len;
  const bool mx = d.is_max ? d.is_max[j] != 0 : false;
  const double s = wave_reduce_range(d.partial + int64_t(j / d.cw) * d.cs + (j % d.cw), 0, d.nblk, d.sb, mx);
  if (threadIdx.x == 0) d.out[j] = s;
}

// sreduce in one launch (one split per segment, at most 8 segments), for up to two reductions: wave w sums
// segment w's blocks exactly as k_wave_reduce's split w does, lane 0 of the block then folds the segment
// values in k_seg_fold's order (nblk = segblk here)
__global__ __launch_bounds__(512) void k_seg_reduce_n(RedDesc d0, RedDesc d1, int nseg) {
  __shared__ double sv[8];
  const int jj = blockIdx.x, w = threadIdx.x >> 6;
  const RedDesc& d = jj < d0.len ? d0 : d1;
  const int j = jj < d0.len ? jj : jj - d0.len;
  const bool mx = d.is_max ? d.is_max[j] != 0 : false;
  if (w < nseg) {
    const double s = wave_reduce_range(d.partial + int64_t(j / d.cw) * d.cs + (j % d.cw), w * d.nblk,
                                       (w + 1) * d.nblk, d.sb, mx);
    if ((threadIdx.x & 63) == 0) sv[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = q < nseg ? sv[q] : 0.0;
#pragma unroll
    for (int wd = 1; wd < 8; wd *= 2)
#pragma unroll
      for (int i = 0; i + wd < 8; i += 2 * wd)
        if (i + wd < nseg) v[i] = mx ? nan_max(v[i], v[i + wd]) : v[i] + v[i + wd];
    d.out[j] = v[0];
  }
}

// Compensated variant: output j folds the (s, c) pairs partial[j * cs + b * sb + {0, 1}] for b in
// [split * span, min(nblk, (split+1) * span)) with comp_merge in a fixed order; final != 0 writes
// s + c to out[j * nsplit + split], else the pair to out[2 (j * nsplit + split) + {0, 1}].
__global__ __launch_bounds__(64) void k_wave_reduce2(const double* __restrict__ partial, int nblk, int span, int64_t sb,
                                                     int64_t cs, int final, double* __restrict__ out, int segblk = 0) {
  const int j = blockIdx.x, split = blockIdx.y, nsplit = gridDim.y, lane = threadIdx.x;
  const double* src = partial + int64_t(j) * cs;
  int b0, b1;
  seg_split_range(split, span, nblk, segblk, b0, b1);
  double s = 0.0, c = 0.0;
  for (int b = b0 + lane; b < b1; b += 64) comp_merge(s, c, src[int64_t(b) * sb], src[int64_t(b) * sb + 1]);
  wave_sum2(s, c);
  if (lane == 0) {
    const int64_t o = int64_t(j) * nsplit + split;
    if (final) out[o] = s + c;
    else { out[2 * o] = s; out[2 * o + 1] = c; }
  }
}

// Segment values -> one value per output, in the fixed pairwise order of gnk.h's gnk_set_segments
// (bottom-up: v[i] += v[i + w] for w = 1, 2, 4, ..., i a multiple of 2w with i + w < n): for a power-of-two
// n this is the balanced binary tree, so a rank holding segments [a, a + n / w) of n folds them into the
// subtree value slab.Comm's rank combine expects.  in[j * nseg + s] -> out[j]; is_max[j]: NaN-propagating max.
constexpr int SEG_MAX = 64;
__device__ __forceinline__ double seg_tree_fold(double (&v)[SEG_MAX], int n, bool mx) {
  for (int w = 1; w < n; w *= 2)
    for (int i = 0; i + w < n; i += 2 * w) v[i] = mx ? nan_max(v[i], v[i + w]) : v[i] + v[i + w];
  return v[0];
}
__global__ __launch_bounds__(64) void k_seg_fold(const double* __restrict__ in, int nseg, int len,
                                                 const int* __restrict__ is_max, double* __restrict__ out) {
  const int j = blockIdx.x * 64 + threadIdx.x;
  if (j >= len) return;
  const bool mx = is_max ? is_max[j] != 0 : false;
  if (nseg <= 8) {
    // the usual case (8 segments per grid): seg_tree_fold's order with the values in registers (the
    // runtime-indexed array of the general form lives in scratch memory)
    double v[8];
#pragma unroll
    for (int sgi = 0; sgi < 8; ++sgi) v[sgi] = sgi < nseg ? in[int64_t(j) * nseg + sgi] : 0.0;
#pragma unroll
    for (int w = 1; w < 8; w *= 2)
#pragma unroll
      for (int i = 0; i + w < 8; i += 2 * w)
        if (i + w < nseg) v[i] = mx ? nan_max(v[i], v[i + w]) : v[i] + v[i + w];
    out[j] = v[0];
    return;
  }
  double v[SEG_MAX];
  for (int sgi = 0; sgi < nseg; ++sgi) v[sgi] = in[int64_t(j) * nseg + sgi];
  out[j] = seg_tree_fold(v, nseg, mx);
}

// out[j] = sum over b of partial[b * stride + j] (mode is_max[j]: NaN-propagating max).
// One block per output; thread t folds b = t, t + 256, ... in order, then a fixed tree:
// the summation order depends only on nblk, so results are bitwise reproducible.
__global__ __launch_bounds__(BLOCK) void k_reduce(const double* __restrict__ partial, int nblk, int len,
                                                  int stride, const int* __restrict__ is_max, double* out) {
  __shared__ double sh[BLOCK];
  const int j = blockIdx.x;
  if (j >= len) return;
  const bool mx = is_max ? is_max[j] != 0 : false;
  double s = 0.0;
  bool any = false;
  for (int b = threadIdx.x; b < nblk; b += BLOCK) {
    const double v = partial[size_t(b) * stride + j];
    s = !any ? v : (mx ? nan_max(s, v) : s + v);
    any = true;
  }
  if (!any) s = mx ? -1.0 : 0.0;     // empty slot: identity (max over |x| >= 0)
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int w = BLOCK / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      const double a = sh[threadIdx.x], bb = sh[threadIdx.x + w];
      sh[threadIdx.x] = mx ? nan_max(a, bb) : a + bb;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = mx ? (sh[0] < 0.0 ? 0.0 : sh[0]) : sh[0];
}

// sum-over-chunks layout used by k_vjp_gemv_t: partial[(z * nblk + b) * KC + j]
__global__ __launch_bounds__(BLOCK) void k_reduce_chunks(const double* __restrict__ partial, int nblk, int k,
                                                         int kct, double* out) {
  for (int jj = blockIdx.x * BLOCK + threadIdx.x; jj < k; jj += gridDim.x * BLOCK) {
    const int z = jj / kct, j = jj % kct;
    const double* p = partial + size_t(z) * nblk * kct + j;
    double s = p[0];
    for (int b = 1; b < nblk; ++b) s += p[size_t(b) * kct];
    out[jj] = s;
  }
}

// ---------------------------------------------------------------- Gram on fp64 MFMA
// v_mfma_f64_16x16x4_f64:  C[16x16] += A[16x4] B[4x16];  lane l holds A[l&15][l>>4],
// B[l>>4][l&15]; C/D reg i of lane l is C[(l>>4) + 4i][l&15] (cdna_hip_programming.md §3).
// For a Gram tile (a, b) over 4 rows: A[i][kk] = W[row kk][16a + i], B[kk][j] = W[row kk][16b + j]
// so lane l supplies W[row l>>4][16a + (l&15)] and W[row l>>4][16b + (l&15)].
__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void pair_ab(int p, int nb, int& a, int& b) {
  a = 0;
  int rem = p;
  while (rem >= nb - a) { rem -= nb - a; ++a; }
  b = a + rem;
}

// W tile rows [e0, e0 + T) in LDS as Wt[t * S + col] (S = KP + 1).
// Pass 1 (rinv == nullptr): W = J V.  Pass 2: W = [J V | r] @ RinvAug (RinvAug kp x kp).
// rowsplit = 1: each wave accumulates all P pair tiles over its quarter of the rows.
// rowsplit = 0: blockIdx.y = pair group; wave w owns pairs grp*4*PPW + w*PPW + q over all rows.
template <int PPW>
__global__ __launch_bounds__(BLOCK) void k_gram(const double* __restrict__ u, const double* __restrict__ V,
                                                int64_t ldv, int k, const double* __restrict__ rinv,
                                                const double* __restrict__ r, Geo geo, Coef c, int T, int logT,
                                                int KP, int P, int rowsplit, int64_t ntiles, int rinv_in_lds,
                                                double* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int S = KP + 1;
  double* Wt = lds;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = KP / 16;
  const int64_t N = geo.N;
  const int64_t nown = geo.nrows * N;
  const int64_t base = int64_t(G) * N;

  int pa[PPW], pb[PPW];
  bool pv[PPW];
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int p = rowsplit ? q : (blockIdx.y * 4 * PPW + wave * PPW + q);
    pv[q] = rowsplit ? (q < P) : (p < P);
    pair_ab(pv[q] ? p : 0, nb, pa[q], pb[q]);
  }
  d4 acc[PPW];
#pragma unroll
  for (int q = 0; q < PPW; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};

  const int rq = rowsplit ? T / 4 : T;
  const int rbeg = rowsplit ? wave * rq : 0;

  // padding columns [K1, KP) stay zero for the whole launch (the pass-2 transform
  // writes zeros there too: RinvAug is zero outside its k(+1) leading block)
  for (int idx = tid; idx < T * S; idx += BLOCK) Wt[idx] = 0.0;
  // RinvAug staged once per launch behind the tile when it fits (the host decides: KP <= 64, and
  // wider bases as long as tile + RinvAug fit the LDS -- a B operand from L2 inside the transform's
  // MFMA chain makes the pass latency-bound)
  double* rinv_lds = (rinv && rinv_in_lds) ? lds + T * S : nullptr;
  if (rinv_lds)
    for (int idx = tid; idx < KP * KP; idx += BLOCK) rinv_lds[idx] = rinv[idx];
  __syncthreads();

  // fill geometry: thread -> (row t, column phase jh); a wave covers 64 consecutive rows
  // of one column, so every load below is a coalesced 512-B wave access.
  const int tpr = BLOCK >> logT;        // threads per row
  const int t = tid & (T - 1);
  const int jh = tid >> logT;
  constexpr int B = 6;                  // columns per batch: 5 B loads in flight per thread

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // Branch-free fill: every load is unconditional (clamped address; ghost rows and
    // the +-1 neighbours are always inside the slab) and masked afterwards with selects,
    // so all 5*B loads of a batch are in flight together (a load under a runtime branch
    // makes hipcc drain vmcnt at the join).
    const int64_t e = (tile << logT) + t;
    const bool valid = e < nown;
    const int64_t i = base + (valid ? e : nown - 1);
    const int64_t iy = (valid ? e : nown - 1) % N;
    const bool hw = iy > 0, he = iy < N - 1;
    const double uu = u[i];
    double dd = 0.0;
    bool have_dd = false;
    for (int j0 = jh; j0 < k; j0 += B * tpr) {
      double vn[B], vw[B], vc[B], ve[B], vs[B];
#pragma unroll
      for (int q = 0; q < B; ++q) {
        const int j = min(j0 + q * tpr, k - 1);
        const double* v = V + j * ldv + i;
        vn[q] = v[-N];
        vw[q] = v[-1];
        vc[q] = v[0];
        ve[q] = v[1];
        vs[q] = v[N];
      }
      if (!have_dd) {
        dd = jdiag(c, uu);
        have_dd = true;
      }
#pragma unroll
      for (int q = 0; q < B; ++q) {
        const int j = j0 + q * tpr;
        const double w = jvp_pt(c, dd, vn[q], hw ? vw[q] : 0.0, hw, vc[q], he ? ve[q] : 0.0, he, vs[q]);
        if (j < k) Wt[t * S + j] = valid ? w : 0.0;
      }
    }
    if (r && (k % tpr) == jh) {
      const double rv = r[i];
      Wt[t * S + k] = valid ? rv : 0.0;
    }
    __syncthreads();
    if (rinv) {
      // in-place W <- W @ RinvAug; column blocks descending so each block reads only
      // not-yet-overwritten blocks a <= cb. Rows split over the 4 waves.
      const double* rv = rinv_lds ? rinv_lds : rinv;
      const int rq4 = T / 4;
      for (int c16 = wave * rq4; c16 < (wave + 1) * rq4; c16 += 16) {
        for (int cb = nb - 1; cb >= 0; --cb) {
          d4 qv = d4{0.0, 0.0, 0.0, 0.0};
          for (int ab = 0; ab <= cb; ++ab) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
              const int kk = ab * 16 + ks * 4 + (lane >> 4);
              const double a = Wt[(c16 + (lane & 15)) * S + kk];
              const double b = rv[kk * KP + cb * 16 + (lane & 15)];
              qv = mfma64(a, b, qv);
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) Wt[(c16 + (lane >> 4) + 4 * i) * S + cb * 16 + (lane & 15)] = qv[i];
        }
      }
      __syncthreads();
    }
    for (int rr = rbeg; rr < rbeg + rq; rr += 4) {
      const double* row = Wt + (rr + (lane >> 4)) * S + (lane & 15);
#pragma unroll
      for (int q = 0; q < PPW; ++q) {
        if (pv[q]) acc[q] = mfma64(row[pa[q] * 16], row[pb[q] * 16], acc[q]);
      }
    }
    __syncthreads();
  }

  // block partial: partial[((grp * gridDim.x + blockIdx.x) * PG + pair_local) * 256 + lane * 4 + i],
  // PG = pairs per group (P when rowsplit, 4 * PPW otherwise)
  const int PG = rowsplit ? P : 4 * PPW;
  double* out = partial + (size_t(blockIdx.y) * gridDim.x + blockIdx.x) * size_t(PG) * 256;
  if (rowsplit) {
    // ((w0 + w1) + w2) + w3 through LDS (reuses the tile; P * 256 <= T * S checked on the host)
    double* red = lds;
    for (int w = 0; w < 4; ++w) {
      if (wave == w) {
#pragma unroll
        for (int q = 0; q < PPW; ++q)
          if (pv[q])
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              double* dst = red + q * 256 + lane * 4 + i;
              *dst = (w == 0) ? acc[q][i] : *dst + acc[q][i];
            }
      }
      __syncthreads();
    }
    for (int idx = tid; idx < P * 256; idx += BLOCK) out[idx] = red[idx];
  } else {
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      if (pv[q]) {
        const int pl = wave * PPW + q;
#pragma unroll
        for (int i = 0; i < 4; ++i) out[size_t(pl) * 256 + lane * 4 + i] = acc[q][i];
      }
    }
  }
}

// Wave-independent Gram pass (KP <= 64).  Every wave streams its own 64-row chunks:
//   lane = row, one basis column per load instruction (the column base is wave-uniform and
//   lives in SGPRs; the three row offsets i-N, i, i+N are 32-bit VGPRs shared by every column,
//   so a load costs no address arithmetic), the J V stencil in registers with the row-edge
//   masks folded into the coefficients, then the wave's private LDS transpose tile
//   [64 rows][KP] -> (pass 2: in-place W <- W RinvAug on MFMA) -> Gram MFMAs accumulating
//   all P pair tiles in registers.  No workgroup barrier inside the chunk loop (a wave's LDS
//   accesses are processed in issue order), so one wave's loads overlap another's MFMAs.

typedef unsigned int u2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double bld(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
}

// Pair tile p of the upper triangle (row-major: (0,0), (0,1), ..., (0,nb-1), (1,1), ...) -> (a, b).
// A fixed-trip-count sum of comparisons, not a data-dependent loop: inside the unrolled tile loops p is
// a constant and the whole index folds away.  (A while loop here was left as a scalar loop in front of
// every Gram MFMA for nb >= 3, serialising each tile's LDS reads behind it.)
constexpr int pair_start(int a, int nb) { return a * nb - a * (a - 1) / 2; }
constexpr int pair_a(int p, int nb) {
  int a = 0;
  for (int i = 1; i < 16; ++i) a += (i < nb && p >= pair_start(i, nb)) ? 1 : 0;
  return a;
}
constexpr int pair_b(int p, int nb) {
  const int a = pair_a(p, nb);
  return a + p - pair_start(a, nb);
}
static_assert(pair_a(0, 7) == 0 && pair_b(6, 7) == 6 && pair_a(7, 7) == 1 && pair_b(7, 7) == 1 &&
              pair_a(27, 7) == 6 && pair_b(27, 7) == 6 && pair_a(12, 7) == 1 && pair_b(12, 7) == 6, "pair_a/b");

__device__ __forceinline__ double dpp_row_shr1(double v) {     // lane l <- lane l-1 of its 16-lane row
  const u2v b = __builtin_bit_cast(u2v, v);
  u2v o;
  o.x = unsigned(__builtin_amdgcn_mov_dpp(int(b.x), 0x111, 0xf, 0xf, true));   // bound_ctrl: row edge -> 0
  o.y = unsigned(__builtin_amdgcn_mov_dpp(int(b.y), 0x111, 0xf, 0xf, true));   // bound_ctrl: row edge -> 0
  return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double dpp_row_shl1(double v) {     // lane l <- lane l+1 of its 16-lane row
  const u2v b = __builtin_bit_cast(u2v, v);
  u2v o;
  o.x = unsigned(__builtin_amdgcn_mov_dpp(int(b.x), 0x101, 0xf, 0xf, true));   // bound_ctrl: row edge -> 0
  o.y = unsigned(__builtin_amdgcn_mov_dpp(int(b.y), 0x101, 0xf, 0xf, true));   // bound_ctrl: row edge -> 0
  return __builtin_bit_cast(double, o);
}

// Wide Gram pass for 5..7 column blocks (KP = 80..112: k = 64..111 on the GNK path), round 3.
// k_gram above stages RinvAug (up to 100 KB) in LDS beside its tile, which leaves one 4-wave workgroup
// per CU: one wave per SIMD runs fill, transform and Gram back to back, so the fp64 pipe idles while a
// tile loads.  Here one 8-wave workgroup per CU walks a 32-point strip down a row range:
//  * fill: thread -> (point pair, column phase); every thread marches its columns down the strip with
//    the centre and south rows in registers (one new 16-B row load per column and step, issued before
//    the step's MFMAs; the north row is the previous centre), the in-row neighbours by DPP row shifts,
//    the strip's outer neighbours by its two edge lanes -- each value leaves HBM once;
//  * transform Y = W P^-1 split over wave pairs by OUTPUT column block (block cb costs cb + 1 k-steps;
//    a greedy split gives each pair <= 2 blocks and equal cost at 7 blocks), the two waves of a pair
//    taking the tile's two 16-row groups; RinvAug's B fragments live in VGPRs for the whole launch and
//    Y goes to a second tile (no in-place hazard);
//  * Gram: each wave pair owns ceil(P / 4) pair tiles, its two waves the two row halves (summed in a
//    fixed order at the end);
//  * jdiag(u) once per point: wave 0 computes the next row's into LDS one step ahead.
// Strips are XCD-major (consecutive workgroups of one XCD take adjacent strips).
constexpr int GX_T = 32;      // points per tile (the strip width)
constexpr int GX_NW = 8;      // waves per workgroup
constexpr int gx_owner(int nb, int cb) {      // wave pair owning transform block cb (greedy by cost cb + 1)
  int load[4] = {0, 0, 0, 0};
  int own = -1;
  for (int c = nb - 1; c >= 0; --c) {
    int w = 0;
    for (int i = 1; i < 4; ++i)
      if (load[i] < load[w]) w = i;
    load[w] += c + 1;
    if (c == cb) own = w;
  }
  return own;
}
constexpr int gx_cb(int nb, int w, int slot) {    // slot-th (0, 1) transform block of wave pair w
  int n = 0;
  for (int cb = nb - 1; cb >= 0; --cb)
    if (gx_owner(nb, cb) == w) {
      if (n == slot) return cb;
      ++n;
    }
  return -1;
}

template <int NB, int WP>
__device__ __forceinline__ void gram_x_wave(const double* __restrict__ u, const double* __restrict__ V, int64_t ldv,
                                            int k, const double* __restrict__ rinv, const double* __restrict__ r,
                                            const Geo& geo, const Coef& c, int64_t rpr, int64_t nitems,
                                            double* __restrict__ lds, double* __restrict__ partial) {
  constexpr int TT = GX_T, KP = 16 * NB, S = KP + 1;
  constexpr int P = NB * (NB + 1) / 2, PPW = (P + 3) / 4;
  constexpr int CA = gx_cb(NB, WP, 0), CBB = gx_cb(NB, WP, 1);
  static_assert(gx_cb(NB, WP, 2) == -1, "at most two transform blocks per wave pair");
  constexpr int NBB = CBB >= 0 ? CBB + 1 : 1;
  constexpr int NTH = 64 * GX_NW;
  constexpr int TPR = NTH / (TT / 2);       // 32 threads (column phases) per point pair
  constexpr int MJ = (KP + TPR - 1) / TPR;  // columns per thread
  const int tid = threadIdx.x, lane = tid & 63;
  const int half = (tid >> 6) & 1;          // this wave's row group (transform) / row half (Gram)
  double* Wt = lds;                         // raw J V (| r) tile, [TT][S]
  double* Yt = lds + TT * S;                // transformed tile (pass 2); pass 1 reads Wt
  double* ddb = lds + 2 * TT * S;           // [2][TT]: jdiag of this step's / the next step's row
  const int64_t N = geo.N;
  const int64_t nstrips = N / TT;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int idx = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;

  // this wave pair's RinvAug B fragments (k-steps of blocks ab <= cb), loaded once (none: CA = -1, a
  // pair without transform work at 2..3 column blocks)
  double rA[CA >= 0 ? CA + 1 : 1][4], rB2[NBB][4];
  if (rinv) {
#pragma unroll
    for (int ab = 0; ab <= CA; ++ab)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) rA[ab][ks] = rinv[(ab * 16 + ks * 4 + (lane >> 4)) * KP + CA * 16 + (lane & 15)];
    if (CBB >= 0) {
#pragma unroll
      for (int ab = 0; ab < NBB; ++ab)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          rB2[ab][ks] = rinv[(ab * 16 + ks * 4 + (lane >> 4)) * KP + CBB * 16 + (lane & 15)];
    }
  }
  d4 acc[PPW];
#pragma unroll
  for (int q = 0; q < PPW; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};

  const int pp = tid & (TT / 2 - 1), jh = tid >> 4;
  const bool ew = pp == 0, ee = pp == TT / 2 - 1;
  const double up = -c.j_lin_up;
  const double* src = rinv ? Yt : Wt;       // what the Gram reads
  const bool rthr = r && (k % TPR) == jh;   // the threads that stage r (column k)

  for (int64_t item = idx; item < nitems; item += nwg) {   // (row range, strip)
    const int64_t x0 = (item / nstrips) * rpr;
    const int64_t x1 = min(geo.nrows, x0 + rpr);
    const int64_t cs = (item % nstrips) * TT;
    const int64_t iy = cs + 2 * pp;
    const bool hw = iy > 0, he = iy + 2 < N;
    const double cw = hw ? c.hm2 : 0.0, ce = he ? c.hm2 : 0.0;   // s + 0*v == s (v finite: in-grid values)
    if (x0 >= x1) continue;
    auto colp = [&](int m, int64_t xr) {
      return V + int64_t(min(jh + TPR * m, k - 1)) * ldv + (G + xr) * N + iy;
    };
    d2 vn[MJ], vc[MJ], vs[MJ];
    double eo[MJ];                          // edge lanes: the strip's outer neighbour in the centre row
#pragma unroll
    for (int m = 0; m < MJ; ++m) {
      const double* q = colp(m, x0);
      vn[m] = *reinterpret_cast<const d2*>(q - N);
      vc[m] = *reinterpret_cast<const d2*>(q);
      vs[m] = *reinterpret_cast<const d2*>(q + N);
      eo[m] = ew ? q[hw ? -1 : 0] : (ee ? q[he ? 2 : 1] : 0.0);
    }
    d2 rc = {0.0, 0.0};
    if (rthr) rc = *reinterpret_cast<const d2*>(r + (G + x0) * N + iy);
    double un = 0.0;                        // threads < TT: u of the next row
    if (tid < TT) {
      ddb[tid] = jdiag(c, u[(G + x0) * N + cs + tid]);
      un = u[(G + x0 + 1) * N + cs + tid];
    }
    __syncthreads();

    for (int64_t x = x0; x < x1; ++x) {
      const int bsel = int((x - x0) & 1);
      const double dn0 = -ddb[bsel * TT + 2 * pp], dn1 = -ddb[bsel * TT + 2 * pp + 1];
#pragma unroll
      for (int m = 0; m < MJ; ++m) {
        const double wl = dpp_row_shr1(vc[m].y);   // lane pp-1's second point
        const double er = dpp_row_shl1(vc[m].x);   // lane pp+1's first point
        const double w = ew ? eo[m] : wl, e = ee ? eo[m] : er;
        // J V with explicit FMAs in the CSR term order, as k_gram_w (the Gram's own summation order
        // already differs from the reference's, so the per-element rounding is not observable)
        double w0 = c.hm2 * vn[m].x;
        w0 = fma(cw, w, w0);
        w0 = fma(dn0, vc[m].x, w0);
        w0 = fma(c.hm2, vc[m].y, w0);
        w0 = fma(up, vs[m].x, w0);
        double w1 = c.hm2 * vn[m].y;
        w1 = fma(c.hm2, vc[m].x, w1);
        w1 = fma(dn1, vc[m].y, w1);
        w1 = fma(ce, e, w1);
        w1 = fma(up, vs[m].y, w1);
        if (jh + TPR * m < k) {
          Wt[(2 * pp) * S + jh + TPR * m] = w0;
          Wt[(2 * pp + 1) * S + jh + TPR * m] = w1;
        }
      }
      if (rthr) {
        Wt[(2 * pp) * S + k] = rc.x;
        Wt[(2 * pp + 1) * S + k] = rc.y;
      }
      if (x + 1 < x1) {                      // march: the next step's rows land under this step's MFMAs
#pragma unroll
        for (int m = 0; m < MJ; ++m) {
          vn[m] = vc[m];
          vc[m] = vs[m];
          const double* q = colp(m, x + 1);
          vs[m] = *reinterpret_cast<const d2*>(q + N);
          eo[m] = ew ? q[hw ? -1 : 0] : (ee ? q[he ? 2 : 1] : 0.0);
        }
        if (rthr) rc = *reinterpret_cast<const d2*>(r + (G + x + 1) * N + iy);
        if (tid < TT) {
          ddb[(bsel ^ 1) * TT + tid] = jdiag(c, un);
          un = u[(G + x + 2) * N + cs + tid];
        }
      }
      __syncthreads();
      if (rinv) {
        // Y[rows of group `half`, cb block] = W[., :16(cb+1)] RinvAug[:16(cb+1), cb block]
        const double* arow = Wt + (half * 16 + (lane & 15)) * S + (lane >> 4);
        if constexpr (CA >= 0) {
          d4 qa = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ab = 0; ab <= CA; ++ab)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) qa = mfma64(arow[ab * 16 + ks * 4], rA[ab][ks], qa);
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) Yt[(half * 16 + (lane >> 4) + 4 * ii) * S + CA * 16 + (lane & 15)] = qa[ii];
        }
        if (CBB >= 0) {
          d4 qb = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ab = 0; ab < NBB; ++ab)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) qb = mfma64(arow[ab * 16 + ks * 4], rB2[ab][ks], qb);
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) Yt[(half * 16 + (lane >> 4) + 4 * ii) * S + CBB * 16 + (lane & 15)] = qb[ii];
        }
        __syncthreads();
      }
#pragma unroll
      for (int rr = 0; rr < TT / 2; rr += 4) {
        const double* row = src + (half * (TT / 2) + rr + (lane >> 4)) * S + (lane & 15);
#pragma unroll
        for (int q = 0; q < PPW; ++q) {
          const int p = WP * PPW + q;
          if (p < P) acc[q] = mfma64(row[pair_a(p, NB) * 16], row[pair_b(p, NB) * 16], acc[q]);
        }
      }
      if (!rinv) __syncthreads();          // the next fill overwrites the tile this Gram read
    }
  }
  // the pair's two row halves summed in a fixed order (half 0 + half 1) through LDS, then
  // partial[(block * 4 PPW + pair) * 256 + lane * 4 + i] (k_gram_reduce, one pair group)
  __syncthreads();
  double* red = lds + WP * PPW * 256;
  if (half == 1) {
#pragma unroll
    for (int q = 0; q < PPW; ++q)
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) red[q * 256 + lane * 4 + ii] = acc[q][ii];
  }
  __syncthreads();
  if (half == 0) {
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const int p = WP * PPW + q;
      if (p < P) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
          partial[(size_t(blockIdx.x) * 4 * PPW + p) * 256 + lane * 4 + ii] = acc[q][ii] + red[q * 256 + lane * 4 + ii];
      }
    }
  }
}

// At 2..4 column blocks two workgroups per CU (4 waves per SIMD, <= 128 VGPRs: NB = 3 / 4 spill 80 / 176 B per
// lane and still run 1.55 / 1.1-1.15x faster than at one workgroup, profiles/round5/gram_x_occupancy_ab.jsonl);
// at 5..7 the spills would cost more than the occupancy gives (k = 64: 27.6 -> 40.5 ms).
template <int NB>
__global__ __launch_bounds__(64 * GX_NW) __attribute__((amdgpu_waves_per_eu(NB <= 4 ? 4 : 1)))
void k_gram_x(const double* __restrict__ u, const double* __restrict__ V,
                                                       int64_t ldv, int k, const double* __restrict__ rinv,
                                                       const double* __restrict__ r, Geo geo, Coef c, int64_t rpr,
                                                       int64_t nitems, double* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  // padding columns [k(+1), KP) of both tiles stay zero (RinvAug is zero outside its leading block)
  for (int idx = threadIdx.x; idx < 2 * GX_T * (16 * NB + 1); idx += 64 * GX_NW) lds[idx] = 0.0;
  __syncthreads();
  // one code path per wave pair: each knows its transform blocks and pair tiles at compile time
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 7)) {
    case 0: gram_x_wave<NB, 0>(u, V, ldv, k, rinv, r, geo, c, rpr, nitems, lds, partial); break;
    case 1: gram_x_wave<NB, 1>(u, V, ldv, k, rinv, r, geo, c, rpr, nitems, lds, partial); break;
    case 2: gram_x_wave<NB, 2>(u, V, ldv, k, rinv, r, geo, c, rpr, nitems, lds, partial); break;
    default: gram_x_wave<NB, 3>(u, V, ldv, k, rinv, r, geo, c, rpr, nitems, lds, partial); break;
  }
}

template <int NB, int BC, int CHT>
__global__ __launch_bounds__(BLOCK) void k_gram_w(const double* __restrict__ u, const double* __restrict__ V,
                                                  int64_t ldv, int k, const double* __restrict__ rinv,
                                                  const double* __restrict__ r, Geo geo, Coef c,
                                                  int64_t nchunks, double* __restrict__ partial) {
  // NB column blocks of 16 (KP = 16 NB), P = NB (NB + 1) / 2 Gram pair tiles; every block / pair
  // loop below is compile-time so the MFMA loops unroll and their LDS reads issue ahead.
  // CHT rows per wave chunk; a lane holds 2 consecutive rows (16-B loads); LPC = CHT/2 lanes
  // cover one column of the chunk, so one load instruction covers CG = 64/LPC columns.
  constexpr int KP = 16 * NB, S = KP + 1, P = NB * (NB + 1) / 2;
  constexpr int LPC = CHT / 2, CG = 64 / LPC;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);    // provably wave-uniform
  const int nwave = blockDim.x >> 6;
  double* Wt = lds + wave * (CHT * S);
  double* rinv_lds = rinv ? lds + nwave * CHT * S : nullptr;
  const int64_t N = geo.N;
  const int64_t nown = geo.nrows * N;
  const int64_t base = int64_t(G) * N;
  const int K1 = k + (r ? 1 : 0);

  d4 acc[P];
#pragma unroll
  for (int q = 0; q < P; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};

  for (int idx = lane; idx < CHT * S; idx += 64) Wt[idx] = 0.0;     // padding columns stay 0
  if (rinv_lds)
    for (int idx = tid; idx < KP * KP; idx += blockDim.x) rinv_lds[idx] = rinv[idx];
  __syncthreads();

  const int64_t nw = int64_t(gridDim.x) * nwave;
  const double up = -c.j_lin_up;
  const int p2 = (lane % LPC) * 2, cg = lane / LPC;

  // row position of the chunk start, advanced incrementally (scalar; no per-chunk division)
  const int64_t ch0 = int64_t(blockIdx.x) * nwave + wave;
  const int64_t step = (nw * CHT) % N;
  int64_t iyb = (ch0 * CHT) % N;
  for (int64_t ch = ch0; ch < nchunks; ch += nw) {
    const int64_t e0 = ch * CHT;
    int64_t iy0 = iyb + p2;
    if (N >= 64) {
      if (iy0 >= N) iy0 -= N;
    } else {
      while (iy0 >= N) iy0 -= N;
    }
    int64_t iy1 = iy0 + 1;
    if (iy1 >= N) iy1 -= N;
    iyb += step;
    if (iyb >= N) iyb -= N;
    const bool val0 = e0 + p2 < nown, val1 = e0 + p2 + 1 < nown;
    // pair start; a fully-invalid tail pair is clamped (its values are discarded); a half-valid
    // pair reads one row into the trailing ghost rows, which always exist
    const int64_t i = base + (val0 ? e0 + p2 : nown - 2);
    const double cw0 = iy0 > 0 ? c.hm2 : 0.0, ce0 = iy0 + 1 < N ? c.hm2 : 0.0;   // s + 0*v == s
    const double cw1 = iy1 > 0 ? c.hm2 : 0.0, ce1 = iy1 + 1 < N ? c.hm2 : 0.0;
    const d2 uu = *reinterpret_cast<const d2*>(u + i);
    const double dn0 = -jdiag(c, uu.x), dn1 = -jdiag(c, uu.y);
    for (int j0 = 0; j0 < k; j0 += CG * BC) {
      d2 vn[BC], vw[BC], vc[BC], ve[BC], vs[BC];
#pragma unroll
      for (int q = 0; q < BC; ++q) {
        const double* cp = V + min(j0 + CG * q + cg, k - 1) * ldv + i;
        vn[q] = *reinterpret_cast<const d2*>(cp - N);
        vw[q] = *reinterpret_cast<const d2*>(cp - 1);    // (i-1, i)
        vc[q] = *reinterpret_cast<const d2*>(cp);
        ve[q] = *reinterpret_cast<const d2*>(cp + 1);    // (i+1, i+2)
        vs[q] = *reinterpret_cast<const d2*>(cp + N);
      }
#pragma unroll
      for (int q = 0; q < BC; ++q) {
        // J V with explicit FMAs (same CSR term order; the Gram's own summation order already
        // differs from the reference's, so the per-element rounding is not observable)
        double s0 = c.hm2 * vn[q].x;
        s0 = fma(cw0, vw[q].x, s0);
        s0 = fma(dn0, vc[q].x, s0);
        s0 = fma(ce0, ve[q].x, s0);
        s0 = fma(up, vs[q].x, s0);
        double s1 = c.hm2 * vn[q].y;
        s1 = fma(cw1, vw[q].y, s1);
        s1 = fma(dn1, vc[q].y, s1);
        s1 = fma(ce1, ve[q].y, s1);
        s1 = fma(up, vs[q].y, s1);
        const int j = j0 + CG * q + cg;
        if (j < k) {
          Wt[p2 * S + j] = val0 ? s0 : 0.0;
          Wt[(p2 + 1) * S + j] = val1 ? s1 : 0.0;
        }
      }
    }
    if (r && cg == 0) {
      const d2 rv = *reinterpret_cast<const d2*>(r + i);
      Wt[p2 * S + k] = val0 ? rv.x : 0.0;
      Wt[(p2 + 1) * S + k] = val1 ? rv.y : 0.0;
    }
    if (rinv) {
      // in place W <- W @ RinvAug, column blocks descending (block cb reads blocks a <= cb only)
#pragma unroll
      for (int c16 = 0; c16 < CHT; c16 += 16) {
#pragma unroll
        for (int cb = NB - 1; cb >= 0; --cb) {
          d4 qv = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ab = 0; ab <= cb; ++ab) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
              if (ab * 16 + ks * 4 < K1) {     // RinvAug rows >= K1 are zero (wave-uniform test)
                const int kk = ab * 16 + ks * 4 + (lane >> 4);
                qv = mfma64(Wt[(c16 + (lane & 15)) * S + kk], rinv_lds[kk * KP + cb * 16 + (lane & 15)], qv);
              }
            }
          }
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) Wt[(c16 + (lane >> 4) + 4 * ii) * S + cb * 16 + (lane & 15)] = qv[ii];
        }
      }
    }
    {
      const double* rowbase = Wt + (lane >> 4) * S + (lane & 15);
#pragma unroll
      for (int r4 = 0; r4 < CHT; r4 += 4) {
        const double* row = rowbase + r4 * S;
        double a[NB];
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) a[bb] = row[bb * 16];
#pragma unroll
        for (int q = 0; q < P; ++q) acc[q] = mfma64(a[pair_a(q, NB)], a[pair_b(q, NB)], acc[q]);
      }
    }
  }

  // block partial = ((w0 + w1) + w2) + ... through LDS, layout [block][pair][lane*4 + i]
  __syncthreads();
  double* red = lds;
  for (int w = 0; w < nwave; ++w) {
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          double* dst = red + q * 256 + lane * 4 + ii;
          *dst = (w == 0) ? acc[q][ii] : *dst + acc[q][ii];
        }
    }
    __syncthreads();
  }
  double* out = partial + size_t(blockIdx.x) * size_t(P) * 256;
  for (int idx = tid; idx < P * 256; idx += blockDim.x) out[idx] = red[idx];
}

// Prefetching chunked Gram pass (KP <= 64; the wide-basis pass, k > 20 on the GNK path).  Same
// 32-row chunks, LDS transpose tile, in-place W <- W RinvAug and Gram MFMAs as k_gram_w, but every
// basis column of the NEXT chunk is loaded while the MFMAs of the current one run: a lane keeps
// all its columns' north / centre / south pairs in registers (3 loads per column instead of 5;
// the in-row neighbours come from the adjacent lanes of the 16-lane DPP row, only the chunk's two
// edge lanes load their outer neighbour), and the loads of chunk c + 1 are issued between the
// stencil of chunk c and its MFMAs.  k_gram_w waits for each column group's loads in turn (SQ
// counters at k = 51: waves waiting 51 % of the time, MFMA busy 27 %).  Same FMA order as
// k_gram_w, so the two kernels give bit-identical Grams.

template <int NB, int CHT>
__global__ __launch_bounds__(BLOCK) void k_gram_wp(
    const double* __restrict__ u, const double* __restrict__ V, int64_t ldv, int k, const double* __restrict__ rinv,
    const double* __restrict__ r, Geo geo, Coef c, int64_t nchunks, double* __restrict__ partial) {
  // a lane holds 2 consecutive rows; LPC lanes per column (a 16-lane DPP row holds one column at
  // CHT = 32, two at CHT = 16: the lanes where a shift would cross a column are the edge lanes)
  constexpr int LPC = CHT / 2, CG = 64 / LPC;
  static_assert(CHT == 16 || CHT == 32, "k_gram_wp: 16- or 32-row chunks");
  constexpr int KP = 16 * NB, S = KP + 1, P = NB * (NB + 1) / 2, NS = KP / CG;   // NS column slots per lane
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwave = blockDim.x >> 6;
  double* Wt = lds + wave * (CHT * S);
  double* rinv_lds = rinv ? lds + nwave * CHT * S : nullptr;
  const int64_t N = geo.N;
  const int64_t nown = geo.nrows * N;
  const int64_t base = int64_t(G) * N;
  const int K1 = k + (r ? 1 : 0);
  __builtin_assume(K1 > 16 * (NB - 1));             // KP = gnk_gram_padded_dim(k, r)

  d4 acc[P];
#pragma unroll
  for (int q = 0; q < P; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  for (int idx = lane; idx < CHT * S; idx += 64) Wt[idx] = 0.0;     // padding columns stay 0
  if (rinv_lds)
    for (int idx = tid; idx < KP * KP; idx += blockDim.x) rinv_lds[idx] = rinv[idx];
  __syncthreads();

  const int64_t nw = int64_t(gridDim.x) * nwave;
  const double up = -c.j_lin_up;
  const int pl = lane % LPC, p2 = pl * 2, cg = lane / LPC;
  const bool edge_w = pl == 0, edge_e = pl == LPC - 1;
  const int eoff = edge_w ? -1 : 2;                 // the edge lane's outer neighbour, relative to its row i

  d2 vn[NS], vc[NS], vs[NS], uu, rv = d2{0.0, 0.0};
  double eo[NS];
  auto issue = [&](int64_t ch) {
    const int64_t e0 = ch * CHT;
    const int64_t i = base + (e0 + p2 < nown ? e0 + p2 : nown - 2);
    uu = *reinterpret_cast<const d2*>(u + i);
    if (r) rv = *reinterpret_cast<const d2*>(r + i);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s * CG < k) {                             // wave-uniform: slot holds at least one column
        const double* cp = V + int64_t(min(s * CG + cg, k - 1)) * ldv + i;
        vn[s] = *reinterpret_cast<const d2*>(cp - N);
        vc[s] = *reinterpret_cast<const d2*>(cp);
        vs[s] = *reinterpret_cast<const d2*>(cp + N);
        eo[s] = (edge_w || edge_e) ? cp[eoff] : 0.0;
      }
    }
  };

  const int64_t ch0 = int64_t(blockIdx.x) * nwave + wave;
  const int64_t step = (nw * CHT) % N;
  int64_t iyb = (ch0 * CHT) % N;
  if (ch0 < nchunks) issue(ch0);
  for (int64_t ch = ch0; ch < nchunks; ch += nw) {
    const int64_t e0 = ch * CHT;
    int64_t iy0 = iyb + p2;
    if (N >= 64) {
      if (iy0 >= N) iy0 -= N;
    } else {
      while (iy0 >= N) iy0 -= N;
    }
    int64_t iy1 = iy0 + 1;
    if (iy1 >= N) iy1 -= N;
    iyb += step;
    if (iyb >= N) iyb -= N;
    const bool val0 = e0 + p2 < nown, val1 = e0 + p2 + 1 < nown;
    const double cw0 = iy0 > 0 ? c.hm2 : 0.0, ce0 = iy0 + 1 < N ? c.hm2 : 0.0;   // s + 0*v == s
    const double cw1 = iy1 > 0 ? c.hm2 : 0.0, ce1 = iy1 + 1 < N ? c.hm2 : 0.0;
    const double dn0 = -jdiag(c, uu.x), dn1 = -jdiag(c, uu.y);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s * CG < k) {
        const double w0 = dpp_row_shr1(vc[s].y), e1 = dpp_row_shl1(vc[s].x);
        const double vw0 = edge_w ? eo[s] : w0, ve1 = edge_e ? eo[s] : e1;
        double s0 = c.hm2 * vn[s].x;
        s0 = fma(cw0, vw0, s0);
        s0 = fma(dn0, vc[s].x, s0);
        s0 = fma(ce0, vc[s].y, s0);
        s0 = fma(up, vs[s].x, s0);
        double s1 = c.hm2 * vn[s].y;
        s1 = fma(cw1, vc[s].x, s1);
        s1 = fma(dn1, vc[s].y, s1);
        s1 = fma(ce1, ve1, s1);
        s1 = fma(up, vs[s].y, s1);
        const int j = s * CG + cg;
        if (j < k) {
          Wt[p2 * S + j] = val0 ? s0 : 0.0;
          Wt[(p2 + 1) * S + j] = val1 ? s1 : 0.0;
        }
      }
    }
    if (r && cg == 0) {
      Wt[p2 * S + k] = val0 ? rv.x : 0.0;
      Wt[(p2 + 1) * S + k] = val1 ? rv.y : 0.0;
    }
    // the next chunk's loads fly while this chunk's MFMAs run
    if (ch + nw < nchunks) issue(ch + nw);
    __builtin_amdgcn_sched_barrier(0);
    if (rinv_lds) {
      // in place W <- W @ RinvAug, column blocks descending (block cb reads blocks a <= cb only)
#pragma unroll
      for (int c16 = 0; c16 < CHT; c16 += 16) {
#pragma unroll
        for (int cb = NB - 1; cb >= 0; --cb) {
          d4 qv = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ab = 0; ab <= cb; ++ab) {
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
              if (ab < NB - 1 || ab * 16 + ks * 4 < K1) {   // RinvAug rows >= K1 are zero
                const int kk = ab * 16 + ks * 4 + (lane >> 4);
                qv = mfma64(Wt[(c16 + (lane & 15)) * S + kk], rinv_lds[kk * KP + cb * 16 + (lane & 15)], qv);
              }
            }
          }
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) Wt[(c16 + (lane >> 4) + 4 * ii) * S + cb * 16 + (lane & 15)] = qv[ii];
        }
      }
    }
    const double* rowbase = Wt + (lane >> 4) * S + (lane & 15);
#pragma unroll
    for (int r4 = 0; r4 < CHT; r4 += 4) {
      const double* row = rowbase + r4 * S;
      double a[NB];
#pragma unroll
      for (int bb = 0; bb < NB; ++bb) a[bb] = row[bb * 16];
#pragma unroll
      for (int q = 0; q < P; ++q) acc[q] = mfma64(a[pair_a(q, NB)], a[pair_b(q, NB)], acc[q]);
    }
  }

  // block partial = ((w0 + w1) + w2) + ... through LDS, layout [block][pair][lane*4 + i]
  __syncthreads();
  double* red = lds;
  for (int w = 0; w < nwave; ++w) {
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          double* dst = red + q * 256 + lane * 4 + ii;
          *dst = (w == 0) ? acc[q][ii] : *dst + acc[q][ii];
        }
    }
    __syncthreads();
  }
  double* out = partial + size_t(blockIdx.x) * size_t(P) * 256;
  for (int idx = tid; idx < P * 256; idx += blockDim.x) out[idx] = red[idx];
}

// Marching Gram pass (N % CHT == 0, k <= 8 CG).  Wave gw owns the vertical strip
// s = gw % nstrips (CHT consecutive grid columns) and walks a contiguous range of grid rows.
// Each lane keeps, for each of its <= 8 basis columns, the values of the current row and the
// row below in registers, so a step loads ONE new row per column (16 B / lane) instead of the
// five stencil loads; the in-row neighbours come from the adjacent lanes (ds_bpermute), only
// the strip's edge lanes load their outer neighbour.  Then the same LDS transpose tile,
// optional in-place W <- W P^-1 and Gram MFMAs as k_gram_w.
template <int NB, int CHT, int MC>
__global__ __launch_bounds__(BLOCK) void k_gram_m(const double* __restrict__ u, const double* __restrict__ V,
                                                  int64_t ldv, int k, const double* __restrict__ rinv,
                                                  const double* __restrict__ r, Geo geo, Coef c,
                                                  double* __restrict__ partial) {
  constexpr int KP = 16 * NB, S = KP + 1, P = NB * (NB + 1) / 2;
  constexpr int LPC = CHT / 2, CG = 64 / LPC;     // <= MC columns per lane
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwave = blockDim.x >> 6;
  double* Wt = lds + wave * (CHT * S);
  double* rinv_lds = rinv ? lds + nwave * CHT * S : nullptr;
  const int64_t N = geo.N;
  const int64_t base = int64_t(G) * N;
  const int K1 = k + (r ? 1 : 0);
  const double up = -c.j_lin_up;

  d4 acc[P];
#pragma unroll
  for (int q = 0; q < P; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  for (int idx = lane; idx < CHT * S; idx += 64) Wt[idx] = 0.0;
  if (rinv_lds)
    for (int idx = tid; idx < KP * KP; idx += blockDim.x) rinv_lds[idx] = rinv[idx];
  __syncthreads();

  const int64_t nw = int64_t(gridDim.x) * nwave;
  const int64_t gw = int64_t(blockIdx.x) * nwave + wave;
  const int64_t nstrips = N / CHT;
  const int64_t nranges = nw / nstrips;
  const int64_t s_id = gw % nstrips, r_id = gw / nstrips;
  const int64_t rpr = (geo.nrows + nranges - 1) / nranges;
  const int64_t jx0 = r_id * rpr, jx1 = min(geo.nrows, jx0 + rpr);
  const int pl = lane % LPC, cg = lane / LPC;
  const int p2 = pl * 2;
  const int64_t iy0 = s_id * CHT + p2;                 // strip is inside one grid row
  const bool hw0 = iy0 > 0, he1 = iy0 + 2 < N;
  const double cw0 = hw0 ? c.hm2 : 0.0, ce1 = he1 ? c.hm2 : 0.0;
  const bool edge_w = pl == 0, edge_e = pl == LPC - 1;

  if (r_id < nranges && jx0 < jx1) {
    // prologue: rows jx0-1 (vn) and jx0 (vc) of every column (ghost rows exist)
    d2 vn[MC], vc[MC];
    int64_t i = base + jx0 * N + iy0;
#pragma unroll
    for (int q = 0; q < MC; ++q) {
      const double* cp = V + min(cg + CG * q, k - 1) * ldv + i;
      vn[q] = *reinterpret_cast<const d2*>(cp - N);
      vc[q] = *reinterpret_cast<const d2*>(cp);
    }
    for (int64_t jx = jx0; jx < jx1; ++jx, i += N) {
      d2 vs[MC];
      double ew[MC], ee[MC];
#pragma unroll
      for (int q = 0; q < MC; ++q) {
        const double* cp = V + min(cg + CG * q, k - 1) * ldv + i;
        vs[q] = *reinterpret_cast<const d2*>(cp + N);
        // outer neighbours of the strip (one lane per column group loads; others get 0 here)
        ew[q] = edge_w ? cp[-1] : 0.0;
        ee[q] = edge_e ? cp[2] : 0.0;
      }
      const d2 uu = *reinterpret_cast<const d2*>(u + i);
      const double dn0 = -jdiag(c, uu.x), dn1 = -jdiag(c, uu.y);
#pragma unroll
      for (int q = 0; q < MC; ++q) {
        // in-row neighbours from the adjacent lanes of the same column group
        double w = __shfl_up(vc[q].y, 1, LPC);
        double e = __shfl_down(vc[q].x, 1, LPC);
        if (edge_w) w = ew[q];
        if (edge_e) e = ee[q];
        double s0 = c.hm2 * vn[q].x;
        s0 = fma(cw0, w, s0);
        s0 = fma(dn0, vc[q].x, s0);
        s0 = fma(c.hm2, vc[q].y, s0);
        s0 = fma(up, vs[q].x, s0);
        double s1 = c.hm2 * vn[q].y;
        s1 = fma(c.hm2, vc[q].x, s1);
        s1 = fma(dn1, vc[q].y, s1);
        s1 = fma(ce1, e, s1);
        s1 = fma(up, vs[q].y, s1);
        const int j = cg + CG * q;
        if (j < k) {
          Wt[p2 * S + j] = s0;
          Wt[(p2 + 1) * S + j] = s1;
        }
        vn[q] = vc[q];
        vc[q] = vs[q];
      }
      if (r && cg == 0) {
        const d2 rv = *reinterpret_cast<const d2*>(r + i);
        Wt[p2 * S + k] = rv.x;
        Wt[(p2 + 1) * S + k] = rv.y;
      }
      if (rinv) {
#pragma unroll
        for (int c16 = 0; c16 < CHT; c16 += 16) {
#pragma unroll
          for (int cb = NB - 1; cb >= 0; --cb) {
            d4 qv = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int ab = 0; ab <= cb; ++ab) {
#pragma unroll
              for (int ks = 0; ks < 4; ++ks) {
                if (ab * 16 + ks * 4 < K1) {
                  const int kk = ab * 16 + ks * 4 + (lane >> 4);
                  qv = mfma64(Wt[(c16 + (lane & 15)) * S + kk], rinv_lds[kk * KP + cb * 16 + (lane & 15)], qv);
                }
              }
            }
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) Wt[(c16 + (lane >> 4) + 4 * ii) * S + cb * 16 + (lane & 15)] = qv[ii];
          }
        }
      }
      const double* rowbase = Wt + (lane >> 4) * S + (lane & 15);
#pragma unroll
      for (int r4 = 0; r4 < CHT; r4 += 4) {
        const double* row = rowbase + r4 * S;
        double a[NB];
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) a[bb] = row[bb * 16];
#pragma unroll
        for (int q = 0; q < P; ++q) acc[q] = mfma64(a[pair_a(q, NB)], a[pair_b(q, NB)], acc[q]);
      }
    }
  }

  __syncthreads();
  double* red = lds;
  for (int w = 0; w < nwave; ++w) {
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          double* dst = red + q * 256 + lane * 4 + ii;
          *dst = (w == 0) ? acc[q][ii] : *dst + acc[q][ii];
        }
    }
    __syncthreads();
  }
  double* out = partial + size_t(blockIdx.x) * size_t(P) * 256;
  for (int idx = tid; idx < P * 256; idx += blockDim.x) out[idx] = red[idx];
}

// ---------------------------------------------------------------- staged Gram pass (LDS-DMA ring)
// One workgroup (8 waves) walks a vertical strip of GS_SW = 128 grid points down a range of grid
// rows.  The raw rows of every basis column, u and r stream global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no VGPR staging) into an R-slot ring (R = 4 or 5, layout at gs_ss below):
// each slot holds one grid row of [V_0 .. V_{k-1}, u, (r)] and a halo block (the strip's outer
// neighbours of every column); with R = 4 the u row runs 3 grid rows ahead (the batched jdiag).
// Wave w owns points 16w .. 16w+15 of each step.  It builds its A fragments of J V straight in
// the MFMA operand layout (lane: point l&15, column block l>>4) from five LDS reads per value,
// transforms them on MFMA with the RinvAug B fragments held in VGPRs (Y = J V P^-1), and --
// because the transform's C/D layout equals the Gram's A/B operand layout -- feeds Y to the Gram
// directly from registers.  Only one 16 x 16 column tile runs on MFMA (f64 MFMA is no faster than
// f64 VALU on MI355X):
//   * k > 16: the k - 16 lead columns' Y[p][t] is broadcast along its 16-lane row (DPP row_newbcast)
//     and every lane accumulates Y[p][t] * Y[p][c] for its column c on VALU;
//   * the r column (RinvAug is the identity there): Y[p][c] * r[p] and r[p]^2 on VALU.
// Those per-lane sums (4 points per step, fixed order) are reduced over the lane groups, waves
// and blocks in a fixed order, like the MFMA tile.
constexpr int GS_SW = 128;
constexpr int GS_NW = 8;
constexpr int GS_TM_MIN = 3;    // first tail (k - 16) whose lead-column sums run on 4x4x4 MFMA (k_gram_s TM)
constexpr int GQ_KMIN = 8;      // first k of the 4x4x4-block staged Gram (k_gram_q)
constexpr int GQ_KMAX = 31;     // last k of k_gram_q (8 column groups; above, the marching / chunked wide passes)
constexpr int GS_KMAX = 20;     // V columns the staged kernel covers (k 21..24 would fit the LDS
                                // ring but the two-block instance then spills past 256 VGPRs)

typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) const void* glb_cvp;

// s_waitcnt with vmcnt(n) and lgkmcnt(0), expcnt untouched (gfx9 encoding)
constexpr unsigned waitcnt_vm_lgkm0(int n) { return unsigned((n & 0xF) | ((n >> 4) << 14) | (0x7 << 4)); }

// lane j of each 16-lane row, broadcast to the row (DPP row_newbcast)
template <int J>
__device__ __forceinline__ double bcast_row(double v) {
  // one v_mov_b64_dpp (DPP64: row_newbcast is its broadcast); mov_dpp: every lane has a valid source,
  // so no "old" value
  return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xF, 0xF, false);
}

// per-lane VALU Gram accumulators of the staged kernel: [tail t < 4 KSL][column block] (NB = 2),
// then r . Y[:, block] per block, then r . r
constexpr int gs_nacc(int nb, int ksl) { return nb == 1 ? 2 : 2 * 4 * ksl + 2 + 1; }

// Ring layout: [ring row q][slot s][point] with slot stride gs_ss(R) doubles and ring-row stride R * gs_ss(R)
// (== 16 mod 32, so a half-wave's fragment reads -- 16 points x 2 columns -- hit 64 distinct banks);
// ring rows q = 0 .. nrow - 1 are V_0 .. V_{k-1}, u, (r), ring row nrow the halo blocks (the strip's
// outer neighbours: column c at 4c + {0, 1 | 2, 3}).  With the slot index a compile-time constant of the
// unrolled step loop, every LDS read is a per-lane base plus an immediate offset.
constexpr int gs_ss(int R) { return R == 4 ? 132 : 144; }

// Software pipeline (one 16-point row step per wave; the barrier at its end also frees a ring slot):
//   step x:  DMA row x+R-1 into the slot of row x-1;
//            Gram of row x from its transform H (issued in step x-1: the MFMA results have had a whole
//            step to land) -- MFMA tile + VALU tail / r;
//            A fragments of row x+1 (rows x .. x+2 of the ring) with dn(x+1) from step x-1;
//            transform of row x+1 -> H (MFMA, consumed in step x+1);  dn(x+2) = -jdiag(u(x+2)).
// Every MFMA accumulates in one chain per output (no register copies, no h0 + h1 adds): the chains of
// the Gram and of the transform interleave, so no MFMA waits on its predecessor.
// Two column blocks (k = 17..20) are laid out lead-first: block 0 = the TAIL = k - 16 lead columns
// 0 .. TAIL-1 (Y there needs only the first 4-column k-step of the triangular transform: 1 MFMA),
// block 1 = the 16 main columns TAIL .. TAIL+15 (every k-step: 5 MFMAs) -- 6 transform MFMAs per
// row step instead of 9 with the 16 columns first (whose 4-column remainder needs all 5 k-steps too).
// The MFMA Gram tile is the main block; the lead columns' sums run on VALU (row_newbcast), or with TM on
// 4x4x4 f64 MFMA blocks (v_mfma_f64_4x4x4_4b: the 16x16 C/D layout of Y -- lane 16p + c: point p, column c --
// is that instruction's B layout with block c >> 2, and its A layout once the lead block's RinvAug fragment
// repeats the lead columns in every 4-lane group; tools/probes/mfma44.hip): lead x main in 4 MFMAs per step,
// lead x lead in one (the four point groups as the four blocks, summed in the scatter).
template <int NB, int L, int KSL, int TAIL, int R, int WPE, bool TM = false>
__global__ __launch_bounds__(64 * GS_NW) __attribute__((amdgpu_waves_per_eu(WPE))) void k_gram_s(const double* __restrict__ u, const double* __restrict__ V,
                                                       int64_t ldv, int k, const double* __restrict__ rinv,
                                                       int ldr, const double* __restrict__ r, Geo geo, Coef cf,
                                                       int64_t rpr, double* __restrict__ partial, int plog) {
  constexpr bool TMF = NB == 2 && TM;                     // lead columns' sums on 4x4x4 MFMA
  constexpr int NACC = TMF ? NB + 3 : gs_nacc(NB, KSL);
  constexpr int TMAX = NB == 2 && !TMF ? 4 * KSL : 0;     // VALU tail accumulator slots of this instance
  constexpr int ER = NB * TMAX, RR = ER + NB;             // accumulator slots of r . Y and r . r
  constexpr int QLM = RR + 1, QLL = RR + 2;               // TMF: lead x main / lead x lead (4x4x4 D layouts)
  constexpr int SS = gs_ss(R);                            // slot stride (doubles)
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t N = geo.N;
  const int nrow = k + 1 + (r ? 1 : 0);             // ring rows: V_0..V_{k-1}, u, (r)
  const int QS = R * SS;                            // ring-row stride
  const int ninst = nrow + 1;                       // DMA instructions per grid row (rows + halo)

  // block -> (row range, strip); consecutive range-major tiles share an XCD (blockIdx % 8),
  // so strip neighbours read each other's halo lines from the same L2
  const int nstrips = int(N / GS_SW);
  const int nwg = gridDim.x, b = blockIdx.x;
  const int idx = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
  const int64_t x0 = int64_t(idx / nstrips) * rpr;
  const int64_t x1 = min(geo.nrows, x0 + rpr);
  const int64_t col0 = int64_t(idx % nstrips) * GS_SW;

  auto nks = [](int ab) constexpr { return ab == NB - 1 ? KSL : 4; };
  // k-steps of output block cb from fragment block ab (NB = 2: the lead block needs the first only)
  auto nkt = [](int cb, int ab) constexpr { return (NB == 2 && cb == 0) ? (ab == 0 ? 1 : 0) : (ab == NB - 1 ? KSL : 4); };
  // RinvAug B fragments [cb][ab][ks] (ordinary loads, before any DMA is in flight)
  const int cl = lane & 15;
  double rB[NB][NB][4];
#pragma unroll
  for (int cb = 0; cb < NB; ++cb)
#pragma unroll
    for (int ab = 0; ab <= cb; ++ab)
#pragma unroll
      for (int ks = 0; ks < nkt(cb, ab); ++ks) {
        const int row = ab * 16 + ks * 4 + (lane >> 4);
        // lead block: columns 0 .. TAIL-1 (the rest of its tile 0; TMF: repeated in every 4-lane group);
        // main: TAIL + cl
        const int lc = TMF ? (cl & 3) : cl;
        if (NB == 2)
          rB[cb][ab][ks] = cb == 0 ? (lc < TAIL ? rinv[row * ldr + lc] : 0.0) : rinv[row * ldr + TAIL + cl];
        else
          rB[cb][ab][ks] = rinv[row * ldr + cl];
        // opaque use: the load retires here, before the first DMA (a VGPR load still counted
        // when a DMA is in flight makes hipcc wait vmcnt(0) at its first use in the step loop)
        asm volatile("" : "+v"(rB[cb][ab][ks]));
      }
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};                  // MFMA tile: columns 0..15 x 0..15
  double ev[NACC];                                  // VALU Gram accumulators (see gs_nacc)
#pragma unroll
  for (int q = 0; q < NACC; ++q) ev[q] = 0.0;

  // This wave's DMA instructions q = wave + 8m (a q past the end re-loads the u row: same bytes,
  // same place): a per-lane source at row 0 and the LDS offset of slot 0 are fixed; a step only adds
  // the row offset and the slot's.
  // EB (R = 4): the u ring row runs 3 grid rows ahead (slot of row y holds u(y + 3)), so every 4th row one
  // jdiag per lane covers 4 rows (lane group g: row x + 2 + g) -- the other rows take their diagonal from
  // that batch by a lane shuffle, not 4 lanes computing the same exp.  (The same batching in the 5-slot ring of
  // the two-block instances, with a run-time batch phase, was bit-identical and 1-4 % slower at k = 17..20:
  // profiles/round6/gram_s_eb5_ab.txt; not kept.  The code below handles both.)
  constexpr bool EB = R == 4;
  const double* dsrc[L];
  int ddst[L];
  bool isu[L];
#pragma unroll
  for (int m = 0; m < L; ++m) {
    int q = wave + GS_NW * m;
    if (q >= ninst) q = k;
    isu[m] = q == k;
    if (q < nrow) {
      const double* rowp = q < k ? V + int64_t(q) * ldv : (q == k ? u : r);
      dsrc[m] = rowp + col0 + 2 * lane;
    } else {
      // halo: lane -> column lane/2, side lane&1.  The domain's outer columns (coefficient 0) load an
      // inside pair instead: the east pair of the last strip would be the 2 elements after a row --
      // past the end of the column on its last ghost row
      const int cc = min(lane >> 1, k - 1);
      const int64_t off = (lane & 1) ? (col0 + GS_SW < N ? col0 + GS_SW : col0 + GS_SW - 2) : (col0 > 0 ? col0 - 2 : 0);
      dsrc[m] = V + int64_t(cc) * ldv + off;
    }
    ddst[m] = q * QS;
  }
  const int64_t rmax = geo.nrows + G - 1;           // last slab row (ghost)
  auto issue_row = [&](int64_t xr, int slot) {     // rows past the slab re-load the last one
    const int64_t roff = (G + min(xr, rmax)) * N;
    const int64_t roffu = (G + min(xr + (EB ? 3 : 0), rmax)) * N;
    double* sbase = lds + slot * SS;
#pragma unroll
    for (int m = 0; m < L; ++m)
      __builtin_amdgcn_global_load_lds((glb_cvp)(dsrc[m] + (isu[m] ? roffu : roff)), (lds_vp)(sbase + ddst[m]), 16,
                                       0, 0);
  };

  // fixed per-lane stencil offsets of every fragment (column j = 16ab + 4ks + l>>4, point e), slot 0
  const int e = wave * 16 + (lane & 15);            // this lane's point in the strip
  const int cq = lane >> 4;
  const double cwm = (col0 + e > 0) ? cf.hm2 : 0.0;
  const double cem = (col0 + e + 1 < N) ? cf.hm2 : 0.0;
  const double up = -cf.j_lin_up;
  const int hq = nrow * QS;                         // the halo ring row
  int fo[NB][4], fw[NB][4], fe[NB][4];
  unsigned fv = 0;                                  // per fragment bit: a V column (else padding)
#pragma unroll
  for (int ab = 0; ab < NB; ++ab)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int j = ab * 16 + ks * 4 + cq;
      const bool isV = j < k;
      const int jr = isV ? j : 0;
      fo[ab][ks] = jr * QS + e;
      fw[ab][ks] = e > 0 ? jr * QS + e - 1 : hq + 4 * jr + 1;             // halo: element -1
      fe[ab][ks] = e < GS_SW - 1 ? jr * QS + e + 1 : hq + 4 * jr + 2;     // halo: element 128
      fv |= unsigned(isV) << (ab * 4 + ks);
    }
  const int ou = k * QS + e;
  const int orr = (k + 1) * QS + wave * 16 + cq;    // r at point 16w + (l>>4) (+ 4i)

  // A fragments of one row (north / centre / south ring slots) with the diagonal dn of that row
  auto stencil = [&](const double* Ln, const double* Lc, const double* Ls, double dn, double (&a)[NB][4]) {
#pragma unroll
    for (int ab = 0; ab < NB; ++ab)
#pragma unroll
      for (int ks = 0; ks < nks(ab); ++ks) {
        const int o = fo[ab][ks];
        const double vn = Ln[o], vw = Lc[fw[ab][ks]], vc = Lc[o], ve = Lc[fe[ab][ks]], vs = Ls[o];
        // J V with explicit FMAs in CSR term order (as k_gram_w).  Only the last fragment can hold
        // columns >= k (padding, coefficients 0): every earlier one is all V columns.
        double sv;
        if (ab == NB - 1 && ks == nks(ab) - 1) {
          const bool isV = (fv >> (ab * 4 + ks)) & 1;
          const double cn = isV ? cf.hm2 : 0.0, cw = isV ? cwm : 0.0, cc = isV ? dn : 0.0;
          const double ce = isV ? cem : 0.0, cs = isV ? up : 0.0;
          sv = cn * vn;
          sv = fma(cw, vw, sv);
          sv = fma(cc, vc, sv);
          sv = fma(ce, ve, sv);
          sv = fma(cs, vs, sv);
        } else {
          sv = cf.hm2 * vn;
          sv = fma(cwm, vw, sv);
          sv = fma(dn, vc, sv);
          sv = fma(cem, ve, sv);
          sv = fma(up, vs, sv);
        }
        a[ab][ks] = sv;
      }
  };
  // H[cb] = A . RinvAug[:, cb block]: one accumulation chain per output block
  auto transform = [&](const double (&a)[NB][4], d4 (&H)[NB]) {
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
      d4 h = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ab = 0; ab <= cb; ++ab)
#pragma unroll
        for (int ks = 0; ks < nkt(cb, ab); ++ks) h = mfma64(a[ab][ks], rB[cb][ab][ks], h);
      H[cb] = h;
    }
  };
  // H[cb][i] = Y[16w + (l>>4) + 4i][col(cb) + (l&15)] (col: 0 for NB = 1; 0 / TAIL for the lead / main
  // block of NB = 2): the MFMA operand of rows 4i..4i+3, and for the VALU part this lane's column at
  // point p = 16w + (l>>4) + 4i
  const int zb = (lane >> 2) & 3;                   // TMF: this lane's 4x4x4 block
  auto gram = [&](const d4 (&Y)[NB], const double* Lr) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = mfma64(Y[NB - 1][i], Y[NB - 1][i], acc);
    if constexpr (TMF) {
      // lead x main: block b = main columns 4b..4b+3, A = the lead columns (repeated), k = the 4 points of group i
#pragma unroll
      for (int i = 0; i < 4; ++i) ev[QLM] = __builtin_amdgcn_mfma_f64_4x4x4f64(Y[0][i], Y[NB - 1][i], ev[QLM], 0, 0, 0);
      // lead x lead: block b takes point group b (lane 16p + 4b + c holds Y[p + 4b][c])
      const double z = zb == 0 ? Y[0][0] : zb == 1 ? Y[0][1] : zb == 2 ? Y[0][2] : Y[0][3];
      ev[QLL] = __builtin_amdgcn_mfma_f64_4x4x4f64(z, z, ev[QLL], 0, 0, 0);
    } else if (NB == 2) {
#pragma unroll
      for (int t = 0; t < TAIL; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double yt;
          switch (t) {
            case 0: yt = bcast_row<0>(Y[0][i]); break;
            case 1: yt = bcast_row<1>(Y[0][i]); break;
            case 2: yt = bcast_row<2>(Y[0][i]); break;
            case 3: yt = bcast_row<3>(Y[0][i]); break;
            case 4: yt = bcast_row<4>(Y[0][i]); break;
            case 5: yt = bcast_row<5>(Y[0][i]); break;
            case 6: yt = bcast_row<6>(Y[0][i]); break;
            default: yt = bcast_row<7>(Y[0][i]); break;
          }
#pragma unroll
          for (int cb = 0; cb < NB; ++cb) ev[t * NB + cb] = fma(yt, Y[cb][i], ev[t * NB + cb]);
        }
      }
    }
    if (r) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double rv = Lr[orr + 4 * i];
#pragma unroll
        for (int cb = 0; cb < NB; ++cb) ev[ER + cb] = fma(rv, Y[cb][i], ev[ER + cb]);
        ev[RR] = fma(rv, rv, ev[RR]);
      }
    }
  };

  // R = 5: row x+4 is issued in step x, row x+3 waited for at its end (one row in flight across
  // each barrier); R = 4: row x+3 is issued in step x and waited for at its end (a smaller ring,
  // so two blocks fit a CU at larger k).  Slot of row xr: (xr - x0 + 1) mod R.
  constexpr int INF = R - 4;                        // rows still in flight at a barrier
  if (x0 < x1) {
    // EB: u of rows x0, x0+1 (the ring's u rows start at x0+2) by ordinary loads before any DMA
    double dn0 = 0.0, dnb = 0.0;                    // dnb: lane group g holds dn of row (batch x) + 2 + g
    if (EB) {
      const int64_t i0 = (G + x0) * N + col0 + e;
      double ua = u[i0], ub = u[i0 + N];
      asm volatile("" : "+v"(ua), "+v"(ub));
      dn0 = -jdiag(cf, ua);
      dnb = -jdiag(cf, ub);                         // every group: dn(x0 + 1), the first step's
    }
#pragma unroll
    for (int s = 0; s < R; ++s) issue_row(x0 - 1 + s, s);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(L * (INF + 1)));   // rows x0-1 .. x0+1 landed
    __builtin_amdgcn_s_barrier();
    d4 H[NB];
    {
      double a[NB][4];
      stencil(lds, lds + SS, lds + 2 * SS, EB ? dn0 : -jdiag(cf, lds[SS + ou]), a);
      transform(a, H);
    }
    double dn = EB ? 0.0 : -jdiag(cf, lds[2 * SS + ou]);        // row x0 + 1
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(L * INF));         // row x0 + 2 landed
    __builtin_amdgcn_s_barrier();
    int bph = 0;                                     // R = 5: batch phase of the next row
    for (int64_t xb = x0; xb < x1; xb += R) {
#pragma unroll
      for (int st = 0; st < R; ++st) {
        const int64_t x = xb + st;
        if (x >= x1) break;
        if (EB) {
          // batch phase of row x, (x - x0) mod 4: compile-time for R = 4, a wave-uniform counter for R = 5
          const int bs = R == 4 ? st : bph;
          bph = (bph + 1) & 3;
          if (bs == 0) {
            dn = __shfl(dnb, 48 + (lane & 15));       // dn(x+1): group 3 of the previous batch
            // the new batch: group g = dn(x+2+g); u(x+2+g) sits in the slot of row x-1+g (slot (x - x0 + g)
            // mod R).  Every wave reads it before any wave's DMA below refills the slot of row x-1 (one more
            // barrier per 4 rows: the u row is DMA'd by one wave, read by all)
            const int sg = (st + cq) % R;        // (x - x0) = st mod R: the ring's slot of row x - 1 + g
            double ug = lds[sg * SS + ou];
            asm volatile("" : "+v"(ug));
            __builtin_amdgcn_s_barrier();
            dnb = -jdiag(cf, ug);
          } else {
            dn = __shfl(dnb, (bs - 1) * 16 + (lane & 15));
          }
        }
        issue_row(x + R - 1, st);                     // into the slot of row x-1
        const double* Lx = lds + ((st + 1) % R) * SS;   // row x
        const double* Lx1 = lds + ((st + 2) % R) * SS;  // row x+1
        const double* Lx2 = lds + ((st + 3) % R) * SS;  // row x+2
        gram(H, Lx);                                  // row x (its r is in slot x)
        if (x + 1 < x1) {
          double a[NB][4];
          stencil(Lx, Lx1, Lx2, dn, a);               // row x+1
          transform(a, H);
          if (!EB) dn = -jdiag(cf, Lx2[ou]);          // row x+2
        }
        __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(L * INF));     // row x+3 landed
        __builtin_amdgcn_s_barrier();
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(0));
  __builtin_amdgcn_s_barrier();

  // block partial = ((w0 + w1) + w2) + ... through LDS:
  //   [0, 256): MFMA tile (lane*4 + i), [256, 256 + 64 NACC): VALU sums (lane * NACC + q)
  constexpr int PL = 256 + 64 * NACC;
  double* red = lds;
  for (int w = 0; w < GS_NW; ++w) {
    if (wave == w) {
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        double* dst = red + lane * 4 + ii;
        *dst = (w == 0) ? acc[ii] : *dst + acc[ii];
      }
#pragma unroll
      for (int q = 0; q < NACC; ++q) {
        double* dst = red + 256 + lane * NACC + q;
        *dst = (w == 0) ? ev[q] : *dst + ev[q];
      }
    }
    __syncthreads();
  }
  double* out = partial + size_t(plog ? idx : b) * PL;     // plog (segments): the logical tile's slot
  if (!plog) {
    for (int t = tid; t < PL; t += blockDim.x) out[t] = red[t];
    return;
  }
  // segments: the scatter's sum over the four lane groups (k_gram_scatter_s, lsum: ((g0 + g1) + g2) + g3)
  // happens here, per workgroup, before any reduction over workgroups, segments or ranks -- summed after
  // them it would not commute with the rank combine.  Group 0's slot gets the sum, groups 1..3 zeros
  // (the scatter's sum then returns it unchanged)
  for (int t = tid; t < PL; t += blockDim.x) {
    if (t < 256) {
      out[t] = red[t];
    } else {
      const int ln = (t - 256) / NACC, q = (t - 256) % NACC, col = ln & 15;
      const double* e = red + 256 + q;
      if (TMF && q == QLM) {       // lead x main (4x4x4 D layout): every lane its own entry
        out[t] = red[t];
      } else if (TMF && q == QLL) {  // lead x lead: the four point-group blocks summed here, into block 0
        const int bl = (ln >> 2) & 3, l0 = ln - 4 * bl;
        out[t] = bl ? 0.0 : ((e[l0 * NACC] + e[(l0 + 4) * NACC]) + e[(l0 + 8) * NACC]) + e[(l0 + 12) * NACC];
      } else
        out[t] = (ln >> 4) ? 0.0 : ((e[col * NACC] + e[(16 + col) * NACC]) + e[(32 + col) * NACC]) + e[(48 + col) * NACC];
    }
  }
}

// ---------------------------------------------------------------- staged Gram pass on 4x4x4 f64 MFMA blocks
// k_gram_s's ring, LDS-DMA pipeline and A fragments, with the transform and the Gram at 4-column granularity on
// v_mfma_f64_4x4x4_4b (512 flops in ~19 cycles: the 16x16x4 form's rate; tools/probes/mfma44.hip maps its
// layouts -- A / B lane 16 k + 4 b + i, D lane 16 i + 4 b + j, b the block).  A stencil fragment of column group
// a (lane 16 q + p: point p = 4 b + i, column 4 a + q) is that instruction's A operand with the four point groups
// as the four blocks, so
//   transform: Y_c = sum_{a <= c} W_a R_ac   -- one 4x4x4 MFMA per (a <= c): the triangle at 4-column granularity,
//              D lane 16 i + 4 b + j = Y[point 4 b + i][column 4 c + j];
//   Gram:      G_cd += Y_c^T Y_d (c <= d)    -- Y_c's D layout read as A is Y_c^T and as B is Y_d, blocks = point
//              groups: one MFMA per group pair, each block a 4-point partial (summed per workgroup below).
// For NG groups that is NG (NG + 1) MFMAs of 19 cycles per 16-point row step, against (transform k-steps + 4)
// 16x16x4 MFMAs of 64 cycles in k_gram_s, with no padding beyond the last 4-column group and no lead/tail split.
// r stays on VALU (r . Y per lane column, r . r).  Per workgroup the lane partials are summed over the point
// groups (and over the points, for r) in a fixed order before any reduction over workgroups, segments or ranks;
// partial[tile][16 NP + 4 NG + 1] holds the group-pair 4x4 blocks, r . Y and r . r (k_gram_scatter_q).
// Instances: 2..4 groups (k = 5..16) on the 4-slot ring, two workgroups per CU; 5 groups (k = 17..20) on 5 slots,
// one per CU; 6..8 groups (k = 21..31, replacing the chunked k_gram_w there) on 4 slots, one per CU, 200-256 VGPRs.
constexpr int gq_np(int ng) { return ng * (ng + 1) / 2; }
constexpr int gq_pl(int ng) { return 16 * gq_np(ng) + 4 * ng + 1; }
__host__ __device__ constexpr int gq_pair(int a, int c) { return c * (c + 1) / 2 + a; }   // a <= c

template <int NG, int L, int R, int WPE>
__global__ __launch_bounds__(64 * GS_NW) __attribute__((amdgpu_waves_per_eu(WPE))) void k_gram_q(
    const double* __restrict__ u, const double* __restrict__ V, int64_t ldv, int k, const double* __restrict__ rinv,
    int ldr, const double* __restrict__ r, Geo geo, Coef cf, int64_t rpr, double* __restrict__ partial, int plog) {
  constexpr int NP = gq_np(NG);
  constexpr int NACC = NP + NG + 1;                 // lane slots: group pairs, r . Y_c, r . r
  constexpr int SS = gs_ss(R);
  constexpr bool EB = R == 4;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t N = geo.N;
  const int nrow = k + 1 + (r ? 1 : 0);             // ring rows: V_0..V_{k-1}, u, (r)
  const int QS = R * SS;
  const int ninst = nrow + 1;

  const int nstrips = int(N / GS_SW);
  const int nwg = gridDim.x, b = blockIdx.x;
  const int idx = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
  const int64_t x0 = int64_t(idx / nstrips) * rpr;
  const int64_t x1 = min(geo.nrows, x0 + rpr);
  const int64_t col0 = int64_t(idx % nstrips) * GS_SW;

  // RinvAug B fragments R_ac (a <= c): lane 16 q + 4 b + j -> RinvAug[4 a + q][4 c + j], every block the same
  double rq[NP];
#pragma unroll
  for (int c = 0; c < NG; ++c)
#pragma unroll
    for (int a = 0; a <= c; ++a) {
      rq[gq_pair(a, c)] = rinv[(4 * a + (lane >> 4)) * ldr + 4 * c + (lane & 3)];
      asm volatile("" : "+v"(rq[gq_pair(a, c)]));   // retired before the first DMA (see k_gram_s)
    }
  double acc[NP], er[NG], err = 0.0;
#pragma unroll
  for (int p = 0; p < NP; ++p) acc[p] = 0.0;
#pragma unroll
  for (int c = 0; c < NG; ++c) er[c] = 0.0;

  const double* dsrc[L];
  int ddst[L];
  bool isu[L];
#pragma unroll
  for (int m = 0; m < L; ++m) {
    int q = wave + GS_NW * m;
    if (q >= ninst) q = k;
    isu[m] = q == k;
    if (q < nrow) {
      const double* rowp = q < k ? V + int64_t(q) * ldv : (q == k ? u : r);
      dsrc[m] = rowp + col0 + 2 * lane;
    } else {
      const int cc = min(lane >> 1, k - 1);
      const int64_t off = (lane & 1) ? (col0 + GS_SW < N ? col0 + GS_SW : col0 + GS_SW - 2) : (col0 > 0 ? col0 - 2 : 0);
      dsrc[m] = V + int64_t(cc) * ldv + off;
    }
    ddst[m] = q * QS;
  }
  const int64_t rmax = geo.nrows + G - 1;
  auto issue_row = [&](int64_t xr, int slot) {
    const int64_t roff = (G + min(xr, rmax)) * N;
    const int64_t roffu = (G + min(xr + (EB ? 3 : 0), rmax)) * N;
    double* sbase = lds + slot * SS;
#pragma unroll
    for (int m = 0; m < L; ++m)
      __builtin_amdgcn_global_load_lds((glb_cvp)(dsrc[m] + (isu[m] ? roffu : roff)), (lds_vp)(sbase + ddst[m]), 16,
                                       0, 0);
  };

  // stencil offsets of column group g (column 4 g + l>>4, point e), slot 0
  const int e = wave * 16 + (lane & 15);
  const int cq = lane >> 4;
  const double cwm = (col0 + e > 0) ? cf.hm2 : 0.0;
  const double cem = (col0 + e + 1 < N) ? cf.hm2 : 0.0;
  const double up = -cf.j_lin_up;
  const int hq = nrow * QS;
  int fo[NG], fw[NG], fe[NG];
  const bool lastv = 4 * (NG - 1) + cq < k;         // the last group's column is a V column (else padding)
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int j = 4 * g + cq;
    const int jr = j < k ? j : 0;
    fo[g] = jr * QS + e;
    fw[g] = e > 0 ? jr * QS + e - 1 : hq + 4 * jr + 1;
    fe[g] = e < GS_SW - 1 ? jr * QS + e + 1 : hq + 4 * jr + 2;
  }
  const int ou = k * QS + e;
  // r at this lane's point in the D layout (lane 16 i + 4 b + j: point 4 b + i)
  const int orq = (k + 1) * QS + wave * 16 + 4 * ((lane >> 2) & 3) + (lane >> 4);

  auto stencil = [&](const double* Ln, const double* Lc, const double* Ls, double dn, double (&a)[NG]) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int o = fo[g];
      const double vn = Ln[o], vw = Lc[fw[g]], vc = Lc[o], ve = Lc[fe[g]], vs = Ls[o];
      double sv;
      if (g == NG - 1) {           // only the last group can hold padding columns (coefficients 0)
        const double cn = lastv ? cf.hm2 : 0.0, cw = lastv ? cwm : 0.0, cc = lastv ? dn : 0.0;
        const double ce = lastv ? cem : 0.0, cs = lastv ? up : 0.0;
        sv = cn * vn;
        sv = fma(cw, vw, sv);
        sv = fma(cc, vc, sv);
        sv = fma(ce, ve, sv);
        sv = fma(cs, vs, sv);
      } else {
        sv = cf.hm2 * vn;
        sv = fma(cwm, vw, sv);
        sv = fma(dn, vc, sv);
        sv = fma(cem, ve, sv);
        sv = fma(up, vs, sv);
      }
      a[g] = sv;
    }
  };
  auto transform = [&](const double (&a)[NG], double (&Y)[NG]) {
#pragma unroll
    for (int c = 0; c < NG; ++c) {
      double h = 0.0;
#pragma unroll
      for (int aa = 0; aa <= c; ++aa) h = __builtin_amdgcn_mfma_f64_4x4x4f64(a[aa], rq[gq_pair(aa, c)], h, 0, 0, 0);
      Y[c] = h;
    }
  };
  auto gram = [&](const double (&Y)[NG], const double* Lr) {
#pragma unroll
    for (int d = 0; d < NG; ++d)
#pragma unroll
      for (int c = 0; c <= d; ++c)
        acc[gq_pair(c, d)] = __builtin_amdgcn_mfma_f64_4x4x4f64(Y[c], Y[d], acc[gq_pair(c, d)], 0, 0, 0);
    if (r) {
      const double rv = Lr[orq];
#pragma unroll
      for (int c = 0; c < NG; ++c) er[c] = fma(rv, Y[c], er[c]);
      err = fma(rv, rv, err);
    }
  };

  constexpr int INF = R - 4;
  if (x0 < x1) {
    double dn0 = 0.0, dnb = 0.0;
    if (EB) {
      const int64_t i0 = (G + x0) * N + col0 + e;
      double ua = u[i0], ub = u[i0 + N];
      asm volatile("" : "+v"(ua), "+v"(ub));
      dn0 = -jdiag(cf, ua);
      dnb = -jdiag(cf, ub);
    }
#pragma unroll
    for (int s = 0; s < R; ++s) issue_row(x0 - 1 + s, s);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(L * (INF + 1)));
    __builtin_amdgcn_s_barrier();
    double Y[NG];
    {
      double a[NG];
      stencil(lds, lds + SS, lds + 2 * SS, EB ? dn0 : -jdiag(cf, lds[SS + ou]), a);
      transform(a, Y);
    }
    double dn = EB ? 0.0 : -jdiag(cf, lds[2 * SS + ou]);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(L * INF));
    __builtin_amdgcn_s_barrier();
    for (int64_t xb = x0; xb < x1; xb += R) {
#pragma unroll
      for (int st = 0; st < R; ++st) {
        const int64_t x = xb + st;
        if (x >= x1) break;
        if (EB) {
          if (st == 0) {
            dn = __shfl(dnb, 48 + (lane & 15));
            const int sg = (st + cq) % R;
            double ug = lds[sg * SS + ou];
            asm volatile("" : "+v"(ug));
            __builtin_amdgcn_s_barrier();
            dnb = -jdiag(cf, ug);
          } else {
            dn = __shfl(dnb, (st - 1) * 16 + (lane & 15));
          }
        }
        issue_row(x + R - 1, st);
        const double* Lx = lds + ((st + 1) % R) * SS;
        const double* Lx1 = lds + ((st + 2) % R) * SS;
        const double* Lx2 = lds + ((st + 3) % R) * SS;
        gram(Y, Lx);
        if (x + 1 < x1) {
          double a[NG];
          stencil(Lx, Lx1, Lx2, dn, a);
          transform(a, Y);
          if (!EB) dn = -jdiag(cf, Lx2[ou]);
        }
        __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(L * INF));
        __builtin_amdgcn_s_barrier();
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(0));
  __builtin_amdgcn_s_barrier();

  // waves summed in order through LDS ([lane * NACC + slot]), then per workgroup: each group pair's 4x4 block
  // over the four point groups ((b0 + b1) + b2) + b3, r . Y_c's column j and r . r over the 16 points (i, b)
  double* red = lds;
  for (int w = 0; w < GS_NW; ++w) {
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        double* dst = red + lane * NACC + q;
        *dst = (w == 0) ? acc[q] : *dst + acc[q];
      }
#pragma unroll
      for (int c = 0; c < NG; ++c) {
        double* dst = red + lane * NACC + NP + c;
        *dst = (w == 0) ? er[c] : *dst + er[c];
      }
      double* dst = red + lane * NACC + NP + NG;
      *dst = (w == 0) ? err : *dst + err;
    }
    __syncthreads();
  }
  constexpr int PL = gq_pl(NG);
  double* out = partial + size_t(plog ? idx : b) * PL;
  for (int t = tid; t < PL; t += blockDim.x) {
    double v = 0.0;
    if (t < 16 * NP) {
      const int p = t >> 4, i = (t >> 2) & 3, j = t & 3;
      const double* e0 = red + (16 * i + j) * NACC + p;
      v = ((e0[0] + e0[4 * NACC]) + e0[8 * NACC]) + e0[12 * NACC];
    } else {
      const int c = (t - 16 * NP) >> 2, j = (t - 16 * NP) & 3;   // c == NG: r . r (lanes j = 0)
      const int q = c < NG ? NP + c : NP + NG;
      for (int i = 0; i < 4; ++i)
        for (int bb = 0; bb < 4; ++bb) v += red[(16 * i + 4 * bb + (c < NG ? j : 0)) * NACC + q];
    }
    out[t] = v;
  }
}

// ---------------------------------------------------------------- VALU Gram pass (k <= 8, with r)
// An f64 MFMA issues no more flops per cycle than f64 VALU FMAs on MI355X (tools/probes), and a
// 16 x 16 MFMA tile spends most of them on padding when the Gram has K + 1 <= 9 columns.  Here the
// whole pass is VALU: every lane owns two adjacent grid points of a 128-point strip and marches
// down a range of rows, loading ONE new row of every column per step (16 B per lane; the row above
// and the current row stay in registers, in-row neighbours come from the adjacent lanes, the
// strip's outer neighbours from the edge lanes' own loads).  Per point it builds J v in the staged
// kernel's FMA order, applies the upper-triangular transform T (wave-uniform: scalar operands),
// appends r, and accumulates the (K + 1)(K + 2) / 2 Gram entries in registers (point 2l, then
// 2l + 1, row by row).  partial[block][NT]: the block's packed upper triangle, row-major
// (row i holds columns i..K), waves summed in order.
template <int K>
__device__ __forceinline__ void gram_v_point(const double (&a)[K], double rv, const double* __restrict__ T, int ldt,
                                             double (&acc)[(K + 1) * (K + 2) / 2]) {
  double y[K + 1];
#pragma unroll
  for (int col = 0; col < K; ++col) {
    double t = a[0] * T[col];
#pragma unroll
    for (int i = 1; i <= col; ++i) t = fma(a[i], T[i * ldt + col], t);
    y[col] = t;
  }
  y[K] = rv;
  int q = 0;
#pragma unroll
  for (int i = 0; i <= K; ++i)
#pragma unroll
    for (int j = i; j <= K; ++j, ++q) acc[q] = fma(y[i], y[j], acc[q]);
}

constexpr int GV_KMAX = 9;      // VALU Gram pass for k <= GV_KMAX (with r); k = 10 measured slower
                                // than the staged kernel (2.20 vs 2.08 ms, 256 VGPRs)
constexpr int GV1_KMIN = 8;     // one point per lane from here (register budget: the two-point k = 8
                                // instance needs 256 VGPRs, one wave per SIMD; 1.40 vs 1.45 ms at 8192^2)
constexpr int GV_SW = 128;           // strip width: 64 lanes x 2 points

template <int K>
__global__ __launch_bounds__(BLOCK) void k_gram_v(const double* __restrict__ u, const double* __restrict__ V,
                                                  int64_t ldv, const double* __restrict__ T, int ldt,
                                                  const double* __restrict__ r, Geo geo, Coef c, int64_t rpr,
                                                  double* __restrict__ partial) {
  constexpr int NT = (K + 1) * (K + 2) / 2;
  __shared__ double red[BLOCK / 64][NT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t N = geo.N;
  const int64_t nstrips = N / GV_SW;
  const int64_t gw = int64_t(blockIdx.x) * (BLOCK / 64) + wave;
  const int64_t x0 = (gw / nstrips) * rpr;
  const int64_t x1 = min(geo.nrows, x0 + rpr);
  const int64_t iy0 = (gw % nstrips) * GV_SW + 2 * lane;
  const double cw0 = iy0 > 0 ? c.hm2 : 0.0, ce1 = iy0 + 2 < N ? c.hm2 : 0.0;
  const double up = -c.j_lin_up;
  const bool edge_w = lane == 0, edge_e = lane == 63;
  const int eoff = edge_w ? -1 : 2;                 // the edge lanes' outer neighbour (others: unused)
  double acc[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) acc[q] = 0.0;
  if (x0 < x1) {
    d2 vn[K], vc[K];
    int64_t i = (G + x0) * N + iy0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      vn[j] = *reinterpret_cast<const d2*>(V + j * ldv + i - N);
      vc[j] = *reinterpret_cast<const d2*>(V + j * ldv + i);
    }
    for (int64_t x = x0; x < x1; ++x, i += N) {
      d2 vs[K];
      double eo[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const double* cp = V + j * ldv + i;
        vs[j] = *reinterpret_cast<const d2*>(cp + N);
        eo[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;     // only the strip's edge lanes load
      }
      const d2 uu = *reinterpret_cast<const d2*>(u + i);
      const d2 rr = *reinterpret_cast<const d2*>(r + i);
      const double dn0 = -jdiag(c, uu.x), dn1 = -jdiag(c, uu.y);
      double a[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        double w = lane_prev(vc[j].y);
        if (edge_w) w = eo[j];
        double s0 = c.hm2 * vn[j].x;
        s0 = fma(cw0, w, s0);
        s0 = fma(dn0, vc[j].x, s0);
        s0 = fma(c.hm2, vc[j].y, s0);
        s0 = fma(up, vs[j].x, s0);
        a[j] = s0;
      }
      gram_v_point<K>(a, rr.x, T, ldt, acc);
#pragma unroll
      for (int j = 0; j < K; ++j) {
        double e = lane_next(vc[j].x);
        if (edge_e) e = eo[j];
        double s1 = c.hm2 * vn[j].y;
        s1 = fma(c.hm2, vc[j].x, s1);
        s1 = fma(dn1, vc[j].y, s1);
        s1 = fma(ce1, e, s1);
        s1 = fma(up, vs[j].y, s1);
        a[j] = s1;
        vn[j] = vc[j];
        vc[j] = vs[j];
      }
      gram_v_point<K>(a, rr.y, T, ldt, acc);
    }
  }
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const double sq = wave_sum(acc[q]);
    if (lane == 0) red[wave][q] = sq;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < NT; q += BLOCK) {
    double sq = red[0][q];
    for (int w = 1; w < BLOCK / 64; ++w) sq += red[w][q];
    partial[size_t(blockIdx.x) * NT + q] = sq;
  }
}

// One-point-per-lane form of k_gram_v (64-point strips, 8-byte loads): half the marching-row registers,
// so K = 9 still runs at two waves per SIMD (1.54 ms vs 2.05 ms for the staged kernel at 8192^2).
template <int K>
__global__ __launch_bounds__(BLOCK) void k_gram_v1(const double* __restrict__ u, const double* __restrict__ V,
                                                   int64_t ldv, const double* __restrict__ T, int ldt,
                                                   const double* __restrict__ r, Geo geo, Coef c, int64_t rpr,
                                                   double* __restrict__ partial) {
  constexpr int NT = (K + 1) * (K + 2) / 2;
  __shared__ double red[BLOCK / 64][NT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t N = geo.N;
  const int64_t nstrips = N / 64;
  const int64_t gw = int64_t(blockIdx.x) * (BLOCK / 64) + wave;
  const int64_t x0 = (gw / nstrips) * rpr;
  const int64_t x1 = min(geo.nrows, x0 + rpr);
  const int64_t iy = (gw % nstrips) * 64 + lane;
  const double cw = iy > 0 ? c.hm2 : 0.0, ce = iy + 1 < N ? c.hm2 : 0.0;
  const double up = -c.j_lin_up;
  const bool edge_w = lane == 0, edge_e = lane == 63;
  const int eoff = edge_w ? -1 : 1;                 // the edge lanes' outer neighbour (others: unused)
  double acc[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) acc[q] = 0.0;
  if (x0 < x1) {
    double vn[K], vc[K];
    int64_t i = (G + x0) * N + iy;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      vn[j] = V[j * ldv + i - N];
      vc[j] = V[j * ldv + i];
    }
    for (int64_t x = x0; x < x1; ++x, i += N) {
      double vs[K], eo[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const double* cp = V + j * ldv + i;
        vs[j] = cp[N];
        eo[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;     // only the strip's edge lanes load
      }
      const double dn = -jdiag(c, u[i]);
      const double rv = r[i];
      double a[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        double w = lane_prev(vc[j]);
        double e = lane_next(vc[j]);
        if (edge_w) w = eo[j];
        if (edge_e) e = eo[j];
        double sv = c.hm2 * vn[j];
        sv = fma(cw, w, sv);
        sv = fma(dn, vc[j], sv);
        sv = fma(ce, e, sv);
        sv = fma(up, vs[j], sv);
        a[j] = sv;
        vn[j] = vc[j];
        vc[j] = vs[j];
      }
      gram_v_point<K>(a, rv, T, ldt, acc);
    }
  }
#pragma unroll
  for (int q = 0; q < NT; ++q) {
    const double sq = wave_sum(acc[q]);
    if (lane == 0) red[wave][q] = sq;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < NT; q += BLOCK) {
    double sq = red[0][q];
    for (int w = 1; w < BLOCK / 64; ++w) sq += red[w][q];
    partial[size_t(blockIdx.x) * NT + q] = sq;
  }
}

// packed upper triangle (K1 columns) -> symmetric G[KP][KP]
__global__ __launch_bounds__(64) void k_gram_scatter_v(const double* __restrict__ red, int K1, int KP,
                                                       double* __restrict__ Gout) {
  // entries outside [0, K1)^2 are zero (written here instead of a memset launch before the scatter)
  for (int idx = threadIdx.x; idx < KP * KP; idx += 64)
    if (idx / KP >= K1 || idx % KP >= K1) Gout[idx] = 0.0;
  for (int i = 0, q = 0; i < K1; ++i)
    for (int j = i; j < K1; ++j, ++q)
      if (q % 64 == int(threadIdx.x)) {
        Gout[i * KP + j] = red[q];
        Gout[j * KP + i] = red[q];
      }
}

// staged-kernel scatter: red = block-summed partials [256 MFMA tile | 64 lanes x NACC]; lane groups
// g = l >> 4 (points) summed in order 0..3.  nb = 1: the MFMA tile holds columns 0..15; nb = 2 (lead
// first, k_gram_s): the VALU sums hold the tail = k - 16 lead columns, the MFMA tile columns
// tail..tail+15; then G[k][c], G[k][k] from the r sums.
__global__ __launch_bounds__(BLOCK) void k_gram_scatter_s(const double* __restrict__ red, int nb, int nacc, int k,
                                                          int has_r, int KP, int tm, double* __restrict__ Gout) {
  const int tail = nb == 2 ? k - 16 : 0;
  const int c0 = tail;                               // first column of the MFMA tile
  const int er = nb == 1 || tm ? 0 : nacc - 3, rr = er + nb;
  const double* ev = red + 256;
  auto lsum = [&](int col_in_block, int q) {
    double s = 0.0;
    for (int g = 0; g < 4; ++g) s += ev[(16 * g + col_in_block) * nacc + q];
    return s;
  };
  // column c of the Gram -> (block, column in block) of the VALU sums
  auto blk = [&](int c) { return c0 ? (c < c0 ? 0 : 1) : (c >> 4); };
  auto cin = [&](int c) { return c0 ? (c < c0 ? c : c - c0) : (c & 15); };
  // entries outside [0, K1)^2 are zero (written here instead of a memset launch before the scatter); the
  // writes below cover [0, K1)^2
  const int K1 = k + has_r;
  for (int idx = blockIdx.x * BLOCK + threadIdx.x; idx < KP * KP; idx += gridDim.x * BLOCK)
    if (idx / KP >= K1 || idx % KP >= K1) Gout[idx] = 0.0;
  for (int idx = blockIdx.x * BLOCK + threadIdx.x; idx < 256 + 24 * 33 + 33; idx += gridDim.x * BLOCK) {
    if (idx < 256) {
      const int lane = idx >> 2, i = idx & 3;
      const int row = (lane >> 4) + 4 * i, col = lane & 15;
      if (c0 + row < k && c0 + col < k && row <= col) {
        Gout[(c0 + row) * KP + c0 + col] = red[idx];
        Gout[(c0 + col) * KP + c0 + row] = red[idx];
      }
    } else if (idx < 256 + 24 * 33) {
      const int t = (idx - 256) / 33, c = (idx - 256) % 33;
      const int trow = c0 ? t : 16 + t;                 // the tail / lead column's Gram row
      // lead = 0: columns c <= 16 + t of row 16 + t;  lead = 1: columns c <= t and the 16 main ones
      const bool want = c0 ? (c <= t || (c >= c0 && c < c0 + 16)) : (c <= 16 + t);
      if (t < tail && want && c < k) {
        // tm: lead x main at lane 16t + (c - c0) of slot rr + 1; lead x lead at lanes 16t + 4b + c of slot
        // rr + 2, the four point-group blocks b summed in order
        const double* e = red + 256;
        const double v = !tm ? lsum(cin(c), t * nb + blk(c))
                         : c >= c0 ? e[(16 * t + c - c0) * nacc + rr + 1]
                                   : ((e[(16 * t + c) * nacc + rr + 2] + e[(16 * t + 4 + c) * nacc + rr + 2]) +
                                      e[(16 * t + 8 + c) * nacc + rr + 2]) + e[(16 * t + 12 + c) * nacc + rr + 2];
        Gout[trow * KP + c] = v;
        Gout[c * KP + trow] = v;
      }
    } else if (has_r) {
      const int c = idx - 256 - 24 * 33;
      if (c < k) {
        const double v = lsum(cin(c), er + blk(c));
        Gout[k * KP + c] = v;
        Gout[c * KP + k] = v;
      } else if (c == k) {
        Gout[k * KP + k] = lsum(0, rr);
      }
    }
  }
}

// G from k_gram_q's reduced partial (gq_pl layout): V-column entries from the group-pair blocks, then r . Y, r . r;
// zero outside [0, k + has_r)^2
__global__ __launch_bounds__(BLOCK) void k_gram_scatter_q(const double* __restrict__ red, int ng, int k, int has_r,
                                                          int KP, double* __restrict__ Gout) {
  const int np = ng * (ng + 1) / 2;
  const int K1 = k + has_r;
  for (int idx = blockIdx.x * BLOCK + threadIdx.x; idx < KP * KP; idx += gridDim.x * BLOCK) {
    const int a = idx / KP, c = idx % KP;
    double v = 0.0;
    if (a < K1 && c < K1) {
      const int lo = min(a, c), hi = max(a, c);
      if (hi < k)            // group pair (lo / 4, hi / 4), entry (lo % 4, hi % 4): one value for both triangles
        v = red[16 * gq_pair(lo >> 2, hi >> 2) + 4 * (lo & 3) + (hi & 3)];
      else if (lo < k)       // r . Y_lo
        v = red[16 * np + lo];
      else                   // r . r
        v = red[16 * np + 4 * ng];
    }
    Gout[idx] = v;
  }
}

// ---------------------------------------------------------------- generic problems (flat vectors)
// Problems other than Bratu keep plain length-n iterate vectors and length-m
// residual vectors; the basis kernels above run on them with a flat geometry (one "row" of n).

// h[j0 + j] partial = V_j . g over a flat vector (the Bratu path fuses this with -J^T r)
template <int VEC, int KCT>
__global__ __launch_bounds__(BLOCK) void k_gemv_t(const double* __restrict__ V, int64_t ldv, int k,
                                                  const double* __restrict__ g, Geo geo, int64_t lr0, int64_t nlr,
                                                  double* __restrict__ partial) {
  __shared__ double sh[(BLOCK / 64) * KCT];
  const int j0 = blockIdx.z * KCT;
  const int kc = max(0, min(KCT, k - j0));
  const int jmax = k - 1;
  double acc[KCT];
#pragma unroll
  for (int j = 0; j < KCT; ++j) acc[j] = 0.0;
  ROW_LOOP_BEGIN(VEC)
  for (int q = 0; q < VEC && iy + q < N; ++q) {
    const double gi = g[li + q];
#pragma unroll
    for (int j = 0; j < KCT; ++j) acc[j] = acc[j] + V[min(j0 + j, jmax) * ldv + li + q] * gi;
  }
  ROW_LOOP_END
  const int nblk = gridDim.x * gridDim.y;
  block_sum_store<KCT>(acc, kc, partial + (size_t(blockIdx.z) * nblk + blockIdx.y * gridDim.x + blockIdx.x) * KCT, sh);
}

// y = A x for a CSR matrix with 32-bit indices; one thread per row, entries in stored order from
// 0 -- scipy's csr_matvec rounding (compiled without FMA contraction).  mode 1: y = -(A x)
// (= (-A) x exactly), mode 2: y = 1 / (A x) (the Jacobi vector 1 / diag(A^T A) from the squared
// entries of A^T and x = 1, summed in the k-ascending order of scipy's csr_matmat)
__global__ __launch_bounds__(BLOCK) void k_csr_spmv(int64_t nrows, const int* __restrict__ indptr,
                                                    const int* __restrict__ indices, const double* __restrict__ data,
                                                    const double* __restrict__ x, double* __restrict__ y, int mode) {
  for (int64_t i = int64_t(blockIdx.x) * BLOCK + threadIdx.x; i < nrows; i += int64_t(gridDim.x) * BLOCK) {
    double s = 0.0;
    for (int jj = indptr[i]; jj < indptr[i + 1]; ++jj) s = s + data[jj] * x[indices[jj]];
    y[i] = mode == 1 ? -s : (mode == 2 ? 1.0 / s : s);
  }
}

// partial of a . b over a flat vector
template <int VEC>
__global__ __launch_bounds__(BLOCK) void k_dot(const double* __restrict__ a, const double* __restrict__ b, Geo geo,
                                               int64_t lr0, int64_t nlr, double* __restrict__ partial) {
  __shared__ double sh[BLOCK / 64 * 2];
  double acc[1] = {0.0}, accc[1] = {0.0};
  ROW_LOOP_BEGIN(VEC)
  for (int q = 0; q < VEC && iy + q < N; ++q) comp_dot(acc[0], accc[0], a[li + q], b[li + q]);
  ROW_LOOP_END
  block_sum2_store<1>(acc, accc, 1, partial + 2 * (blockIdx.y * gridDim.x + blockIdx.x), sh);
}

// Gram of [W P^-1 | r] for a materialised W (k columns of length m, column stride ldw):
// 16-row chunks per wave, A fragments loaded in the f64 MFMA operand layout, the transform on
// MFMA with the RinvAug B fragments in VGPRs and the transformed rows fed to the Gram MFMAs from
// registers (as k_gram_s); all NB (NB + 1) / 2 pair tiles on MFMA.  Block partials [block][P][256].
template <int NB>
__global__ __launch_bounds__(BLOCK) void k_flat_gram(const double* __restrict__ W, int64_t ldw, int k,
                                                     const double* __restrict__ rinv, int ldr,
                                                     const double* __restrict__ r, int64_t m,
                                                     double* __restrict__ partial) {
  constexpr int P = NB * (NB + 1) / 2;
  __shared__ double red[P * 256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double rB[NB][NB][4];
#pragma unroll
  for (int cb = 0; cb < NB; ++cb)
#pragma unroll
    for (int ab = 0; ab <= cb; ++ab)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) rB[cb][ab][ks] = rinv[(ab * 16 + ks * 4 + (lane >> 4)) * ldr + cb * 16 + (lane & 15)];
  d4 acc[P];
#pragma unroll
  for (int q = 0; q < P; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
  const int64_t nchunk = (m + 15) / 16;
  const int64_t nw = int64_t(gridDim.x) * (BLOCK / 64);
  for (int64_t c = int64_t(blockIdx.x) * (BLOCK / 64) + wave; c < nchunk; c += nw) {
    const int64_t row = c * 16 + (lane & 15);
    const bool rv = row < m;
    const int64_t rowc = rv ? row : m - 1;
    double a[NB][4];
#pragma unroll
    for (int ab = 0; ab < NB; ++ab)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int j = ab * 16 + ks * 4 + (lane >> 4);
        const double* src = j < k ? W + int64_t(j) * ldw : r;   // a valid row always (clamped)
        const double v = (r || j < k) ? src[rowc] : 0.0;
        a[ab][ks] = (rv && (j < k || (r && j == k))) ? v : 0.0;
      }
    d4 qv[NB];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
      qv[cb] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ab = 0; ab <= cb; ++ab)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) qv[cb] = mfma64(a[ab][ks], rB[cb][ab][ks], qv[cb]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < P; ++q) acc[q] = mfma64(qv[pair_a(q, NB)][i], qv[pair_b(q, NB)][i], acc[q]);
  }
  for (int w = 0; w < BLOCK / 64; ++w) {
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
          double* dst = red + q * 256 + lane * 4 + ii;
          *dst = (w == 0) ? acc[q][ii] : *dst + acc[q][ii];
        }
    }
    __syncthreads();
  }
  double* out = partial + size_t(blockIdx.x) * size_t(P) * 256;
  for (int t = tid; t < P * 256; t += BLOCK) out[t] = red[t];
}

// Flat Gram for bases wider than k_flat_gram's four 16-column blocks (generic problems, SURVEY f1:
// the reference grows the basis to max_iter - 1 columns without restart, ref:krylow.py:72-73).  Two
// plain passes, both deterministic:
//   Y[j][i] = sum_{l <= j} W[l][i] RinvAug[l][j]   (l ascending; Y[k] = r, padding columns 0)
//   Gout[a][b] = Gout[b][a] = sum_i Y[a][i] Y[b][i]   (one block per pair a <= b, compensated sums)
// The generic path's sizes are small (m residuals of a user problem): these run once per pass.
__global__ __launch_bounds__(BLOCK) void k_flat_ytrans(const double* __restrict__ W, int64_t ldw, int k,
                                                       const double* __restrict__ rinv, int ldr,
                                                       const double* __restrict__ r, int64_t m, int kp,
                                                       double* __restrict__ Y) {
  const int j = blockIdx.y;
  for (int64_t i = int64_t(blockIdx.x) * BLOCK + threadIdx.x; i < m; i += int64_t(gridDim.x) * BLOCK) {
    double y = 0.0;
    if (j < k) {
      for (int l = 0; l <= j; ++l) y = fma(W[int64_t(l) * ldw + i], rinv ? rinv[int64_t(l) * ldr + j] : (l == j), y);
    } else if (j == k && r) {
      y = r[i];
    }
    Y[int64_t(j) * m + i] = y;
  }
}

__global__ __launch_bounds__(BLOCK) void k_flat_syrk(const double* __restrict__ Y, int64_t m, int kp,
                                                     double* __restrict__ Gout) {
  __shared__ double sh[BLOCK / 64 * 2];
  // pair index -> (a, b), a <= b, row-major over the upper triangle
  int p = blockIdx.x, a = 0;
  while (p >= kp - a) { p -= kp - a; ++a; }
  const int b = a + p;
  double s[1] = {0.0}, c[1] = {0.0};
  const double* ya = Y + int64_t(a) * m;
  const double* yb = Y + int64_t(b) * m;
  for (int64_t i = threadIdx.x; i < m; i += BLOCK) comp_dot(s[0], c[0], ya[i], yb[i]);
  double out[2];
  block_sum2_store<1>(s, c, 1, out, sh);
  if (threadIdx.x == 0) {
    const double v = out[0] + out[1];
    Gout[a * kp + b] = v;
    Gout[b * kp + a] = v;
  }
}

// Sum Gram partials over blocks (block order) and scatter into G[KP][KP] (symmetric).
// scatter the reduced pair tiles (red[pair * 256 + lane * 4 + i]) into symmetric G[KP][KP]
__global__ __launch_bounds__(BLOCK) void k_gram_scatter(const double* __restrict__ red, int P, int KP,
                                                        double* __restrict__ Gout) {
  const int nb = KP / 16;
  for (int idx = blockIdx.x * BLOCK + threadIdx.x; idx < P * 256; idx += gridDim.x * BLOCK) {
    const int p = idx >> 8, li = idx & 255, lane = li >> 2, i = li & 3;
    int a, bb;
    pair_ab(p, nb, a, bb);
    const int row = a * 16 + (lane >> 4) + 4 * i;
    const int col = bb * 16 + (lane & 15);
    if (a != bb || row <= col) {
      Gout[row * KP + col] = red[idx];
      Gout[col * KP + row] = red[idx];
    }
  }
}

__global__ __launch_bounds__(BLOCK) void k_gram_reduce(const double* __restrict__ partial, int nblk, int P,
                                                       int PG, int KP, double* __restrict__ Gout) {
  const int nb = KP / 16;
  for (int idx = blockIdx.x * BLOCK + threadIdx.x; idx < P * 256; idx += gridDim.x * BLOCK) {
    const int p = idx >> 8, li = idx & 255, lane = li >> 2, i = li & 3;
    const int grp = p / PG, pl = p % PG;
    const double* src = partial + (size_t(grp) * nblk * PG + pl) * 256 + li;
    double s = src[0];
    for (int b = 1; b < nblk; ++b) s += src[size_t(b) * PG * 256];
    int a, bb;
    pair_ab(p, nb, a, bb);
    const int row = a * 16 + (lane >> 4) + 4 * i;
    const int col = bb * 16 + (lane & 15);
    if (a != bb || row <= col) {
      Gout[row * KP + col] = s;
      Gout[col * KP + row] = s;
    }
  }
}

// ---------------------------------------------------------------- least squares on the device
// One preconditioned CholeskyQR solve of the GNK step (lls.py, ref:gauss_newton_krylow.py:16-36)
// from a Gram of [J V T | r] that is already summed over ranks: one wave, k <= LS_KMAX.
//   rescale: divide row and then column k-1 of G by s = sqrt(G[k-1][k-1]), P[k-1][k-1] = s
//   G[:k, :k] = Ry^T Ry (unblocked Cholesky, dpotf2's left-looking order);  z = Ry^-T G[:k, k];
//   R = Ry P;  d = -R^-1 z (dtrsv's column order);  jdd = ||R d||^2;
//   e_try = e + s_dd * d  (the first Armijo trial point's stored coefficients).
// out: [status, jdd, s, d (k), R (k x k), Ry (k x k), R^-1 (k x k)]; status 0 = ok, 1 = G[:k, :k] not
// numerically SPD.  (R^-1 feeds the next step's transform, k_lls_next.)
constexpr int LS_KMAX = 32;
constexpr int LS_LD = LS_KMAX + 1;

__global__ __launch_bounds__(64) void k_lls(const double* __restrict__ Gm, int kp, int k, const double* __restrict__ P,
                                            int rescale, const double* __restrict__ sdd,
                                            const double* __restrict__ e, double* __restrict__ out,
                                            double* __restrict__ etry) {
  __shared__ double g[LS_LD][LS_LD + 1];
  __shared__ double p[LS_KMAX][LS_LD];
  __shared__ double ry[LS_KMAX][LS_LD];
  __shared__ double rr[LS_KMAX][LS_LD];
  __shared__ double sv[LS_KMAX];
  __shared__ int bad;
  const int l = threadIdx.x;
  const int k1 = k + 1;
  for (int idx = l; idx < k1 * k1; idx += 64) g[idx / k1][idx % k1] = Gm[(idx / k1) * kp + idx % k1];
  for (int idx = l; idx < k * k; idx += 64) p[idx / k][idx % k] = P[idx];
  if (l == 0) bad = 0;
  __syncthreads();
  double s = 1.0;
  if (rescale) {
    const double s2 = g[k - 1][k - 1];
    __syncthreads();      // every thread holds s2 before any thread rescales row k-1 (LDS race)
    if (isfinite(s2) && s2 > 0.0) {
      s = sqrt(s2);
      if (l < k1) g[k - 1][l] = g[k - 1][l] / s;          // lls.py: Gp[k-1, :] /= s
      __syncthreads();
      if (l < k1) g[l][k - 1] = g[l][k - 1] / s;          //         Gp[:, k-1] /= s
      if (l == 0) p[k - 1][k - 1] = s;
      __syncthreads();
    }
  }
  // Cholesky, upper: row j from the rows above it
  for (int j = 0; j < k; ++j) {
    double t = 0.0;
    if (l >= j && l < k) {
      t = g[j][l];
      for (int i = 0; i < j; ++i) t = t - ry[i][j] * ry[i][l];
    }
    if (l == j) {
      if (!(t > 0.0)) bad = 1;
      ry[j][j] = sqrt(t);
    }
    __syncthreads();
    if (l > j && l < k) ry[j][l] = t / ry[j][j];
    if (l < j) ry[j][l] = 0.0;
    __syncthreads();
  }
  // z = Ry^-T G[:k, k] (forward substitution, subtractions in row order)
  double b = (l < k) ? g[l][k] : 0.0;
  for (int j = 0; j < k; ++j) {
    if (l == j) sv[j] = b / ry[j][j];
    __syncthreads();
    if (l > j && l < k) b = b - ry[j][l] * sv[j];
  }
  __syncthreads();
  // R = Ry P (upper x upper)
  if (l < k) {
    for (int i = 0; i < k; ++i) {
      double a = 0.0;
      for (int m = i; m <= l; ++m) a = a + ry[i][m] * p[m][l];
      rr[i][l] = (i <= l) ? a : 0.0;
    }
  }
  __syncthreads();
  // x = R^-1 z, column-oriented back substitution; d = -x
  double xv = (l < k) ? sv[l] : 0.0;
  __syncthreads();
  for (int j = k - 1; j >= 0; --j) {
    if (l == j) sv[j] = xv / rr[j][j];
    __syncthreads();
    if (l < j) xv = xv - sv[j] * rr[l][j];
    __syncthreads();
  }
  const double d = (l < k) ? -sv[l] : 0.0;
  // jdd = sum_i (R d)_i^2 (lane i: row i; summed by lane 0 in row order)
  __shared__ double rd2[LS_KMAX];
  if (l < k) {
    double a = 0.0;
    for (int c = l; c < k; ++c) a = a + rr[l][c] * (-sv[c]);
    rd2[l] = a * a;
  }
  __syncthreads();
  if (l == 0) {
    double jdd = 0.0;
    for (int i = 0; i < k; ++i) jdd = jdd + rd2[i];
    out[0] = bad ? 1.0 : 0.0;
    out[1] = jdd;
    out[2] = s;
  }
  if (l < k) {
    out[3 + l] = d;
    etry[l] = e[l] + sdd[l] * d;
    for (int i = 0; i < k; ++i) {
      out[3 + k + i * k + l] = rr[i][l];
      out[3 + k + k * k + i * k + l] = ry[i][l];
    }
    // column l of R^-1 (back substitution on e_l); rows below l are zero.  Loops unrolled to LS_KMAX so
    // every index into xc is a compile-time constant: xc lives in registers (a runtime-indexed xc went to
    // scratch memory, 272 B per lane, and the solve took 27 us on average at the bench's k)
    double* rinv = out + 3 + k + 2 * k * k;
    double xc[LS_KMAX];
#pragma unroll
    for (int i = LS_KMAX - 1; i >= 0; --i) {
      double a = (i == l) ? 1.0 : 0.0;
#pragma unroll
      for (int m = i + 1; m < LS_KMAX; ++m)
        if (m <= l) a = a - rr[i][m] * xc[m];           // m <= l < k: the same subtractions in the same order
      xc[i] = (i < k && i <= l) ? a / rr[i][i] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < LS_KMAX; ++i)
      if (i < k) rinv[i * k + l] = xc[i];
  }
}

// k_lls on 32 x 32 threads (16 waves): thread (i, l) = (t / 32, t % 32) owns entry (i, l) of the
// factorisation's upper triangles -- the same solve with the same IEEE operations in the same order as
// k_lls (tests/test_gpu_lls_regs.py compares them bit for bit), but the O(k^3) parts run one entry per
// thread: the Cholesky right-looking (entry (i, l) subtracts ry[j][i] ry[j][l] for j = 0, 1, .. exactly as
// k_lls's left-looking dot product does, the pivot row per step), R = Ry P one dot product per entry, R^-1
// one row per step.  Only the two triangular solves of the step itself stay sequential (k barriers each).
// k_lls (one wave, column per lane) spends 5 us at k = 1 .. 52 us at k = 20 in dependent chains through LDS
// (a register form of it, v_readlane instead of LDS, measured the same: ~7 k dependent instructions at
// k = 20); this form: 4 us .. 28 us, ~6 barriers of 16 waves per column.
__global__ __launch_bounds__(1024) void k_lls_2d(const double* __restrict__ Gm, int kp, int k,
                                                 const double* __restrict__ P, int rescale,
                                                 const double* __restrict__ sdd, const double* __restrict__ e,
                                                 double* __restrict__ out, double* __restrict__ etry) {
  __shared__ double g[LS_LD][LS_LD + 1];
  __shared__ double pm[LS_KMAX][LS_LD];
  __shared__ double ry[LS_KMAX][LS_LD];
  __shared__ double rr[LS_KMAX][LS_LD];
  __shared__ double xm[LS_KMAX][LS_LD];
  __shared__ double sv[LS_KMAX], rd2[LS_KMAX];
  __shared__ int bad;
  const int t = threadIdx.x, i = t >> 5, l = t & 31;
  const int k1 = k + 1;
  for (int idx = t; idx < k1 * k1; idx += 1024) g[idx / k1][idx % k1] = Gm[(idx / k1) * kp + idx % k1];
  for (int idx = t; idx < k * k; idx += 1024) pm[idx / k][idx % k] = P[idx];
  if (t == 0) bad = 0;
  __syncthreads();
  double s = 1.0;
  if (rescale) {
    const double s2 = g[k - 1][k - 1];
    __syncthreads();      // every thread holds s2 before any thread rescales row k-1 (LDS race)
    if (isfinite(s2) && s2 > 0.0) {
      s = sqrt(s2);
      if (t < k1) g[k - 1][t] = g[k - 1][t] / s;          // lls.py: Gp[k-1, :] /= s
      __syncthreads();
      if (t < k1) g[t][k - 1] = g[t][k - 1] / s;          //         Gp[:, k-1] /= s
      if (t == 0) pm[k - 1][k - 1] = s;
      __syncthreads();
    }
  }
  // Cholesky, upper
  double gv = (i <= l && l < k) ? g[i][l] : 0.0;
  for (int j = 0; j < k; ++j) {
    if (i == j && l == j) {
      if (!(gv > 0.0)) bad = 1;
      ry[j][j] = sqrt(gv);
    }
    __syncthreads();
    if (i == j && l < k) {
      if (l > j) ry[j][l] = gv / ry[j][j];
      else if (l < j) ry[j][l] = 0.0;
    }
    __syncthreads();
    if (i > j && i <= l && l < k) gv = gv - ry[j][i] * ry[j][l];
  }
  // z = Ry^-T G[:k, k] (forward substitution, subtractions in row order)
  double b = (t < k) ? g[t][k] : 0.0;
  for (int j = 0; j < k; ++j) {
    if (t == j) sv[j] = b / ry[j][j];
    __syncthreads();
    if (t > j && t < k) b = b - ry[j][t] * sv[j];
  }
  // R = Ry P, one entry per thread (m ascending)
  if (i < k && l < k) {
    double a = 0.0;
    for (int m = i; m <= l; ++m) a = a + ry[i][m] * pm[m][l];
    rr[i][l] = (i <= l) ? a : 0.0;
  }
  __syncthreads();
  // x = R^-1 z, column-oriented back substitution; d = -x
  double xv = (t < k) ? sv[t] : 0.0;
  __syncthreads();
  for (int j = k - 1; j >= 0; --j) {
    if (t == j) sv[j] = xv / rr[j][j];
    __syncthreads();
    if (t < j) xv = xv - sv[j] * rr[t][j];
  }
  __syncthreads();
  const double d = (t < k) ? -sv[t] : 0.0;
  if (t < k) {
    double a = 0.0;
    for (int c = t; c < k; ++c) a = a + rr[t][c] * (-sv[c]);
    rd2[t] = a * a;
  }
  // R^-1, one row per step (rows descending): X[r][l] = (delta_rl - sum_{m=r+1..l} R[r][m] X[m][l]) / R[r][r]
  for (int r = k - 1; r >= 0; --r) {
    if (i == r && l < k) {
      double a = (r == l) ? 1.0 : 0.0;
      for (int m = r + 1; m <= l; ++m) a = a - rr[r][m] * xm[m][l];
      xm[r][l] = (r <= l) ? a / rr[r][r] : 0.0;
    }
    __syncthreads();
  }
  if (t == 0) {
    double jdd = 0.0;
    for (int q = 0; q < k; ++q) jdd = jdd + rd2[q];
    out[0] = bad ? 1.0 : 0.0;
    out[1] = jdd;
    out[2] = s;
  }
  if (t < k) {
    out[3 + t] = d;
    etry[t] = e[t] + sdd[t] * d;
  }
  if (i < k && l < k) {
    out[3 + k + i * k + l] = rr[i][l];
    out[3 + k + k * k + i * k + l] = ry[i][l];
    out[3 + k + 2 * k * k + i * k + l] = xm[i][l];
  }
}

// The next GNK step's least-squares inputs, on the device (speculative enqueue; lls.py / krylow.py
// bookkeeping restated): this step solved over k columns (the last one pending if `pending`), its
// first trial was accepted (t = 1) and the basis update appended a pending column with raw products
// h = pack[3:3+k] (rank-summed); pack[1] = sum w^2 of this step's pending column.
//   sc' = [sc[:k-1], 1 / ||w||] (pending) or sc[:k];  hh' = sc' (sc' h);
//   R_true = R with its last column / ||w|| (pending);  P' = blockdiag(R_true, 1);
//   T' = [[diag(sc') D R^-1, -hh'], [0, 1]] (+ the r column), D = diag(1, .., ||w||)  (= M' P'^-1);
//   sdd' = [sc', 1];  e' = [e_try, 0].
__global__ __launch_bounds__(256) void k_lls_next(int k, int pending, const double* __restrict__ out,
                                                 const double* __restrict__ etry, const double* __restrict__ pack,
                                                 const double* __restrict__ sc, int kpn, double* __restrict__ T,
                                                 double* __restrict__ Pn, double* __restrict__ sddn,
                                                 double* __restrict__ en, double* __restrict__ hhn,
                                                 double* __restrict__ scn) {
  const int l = threadIdx.x;
  const int kn = k + 1;
  const double* R = out + 3 + k;
  const double* rinv = out + 3 + k + 2 * k * k;
  const double nrm = pending ? sqrt(pack[1]) : 1.0;
  for (int j = l; j < k; j += 256) {
    const double scj = (pending && j == k - 1) ? 1.0 / nrm : sc[j];
    scn[j] = scj;
    sddn[j] = scj;
    en[j] = etry[j];
    hhn[j] = scj * (scj * pack[3 + j]);
  }
  if (l == 0) {
    sddn[k] = 1.0;
    en[k] = 0.0;
  }
  __syncthreads();
  for (int idx = l; idx < kpn * kpn; idx += 256) {
    const int i = idx / kpn, j = idx % kpn;
    double t = 0.0;
    if (i < k && j < k) {
      const double di = (pending && i == k - 1) ? nrm : 1.0;
      t = (scn[i] * di) * rinv[i * k + j];
    } else if (i < k && j == k) {
      t = -hhn[i];
    } else if (i == j && i <= kn) {
      t = 1.0;                                      // the pending column (i = k) and r (i = k + 1)
    }
    T[idx] = t;
  }
  for (int idx = l; idx < kn * kn; idx += 256) {
    const int i = idx / kn, j = idx % kn;
    double pv = 0.0;
    if (i < k && j < k) pv = (pending && j == k - 1) ? R[i * k + j] / nrm : R[i * k + j];
    else if (i == k && j == k) pv = 1.0;
    Pn[idx] = pv;
  }
}

// ---------------------------------------------------------------- probes (tooling)
__global__ void k_probe_mfma(double* out, int iters) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  for (int i = 0; i < iters; ++i) {
    c0 = mfma64(a, b, c0);
    c1 = mfma64(b, a, c1);
    c2 = mfma64(a, a, c2);
    c3 = mfma64(b, b, c3);
  }
  const d4 s = c0 + c1 + c2 + c3;
  if (s[0] == 12345.0) out[threadIdx.x] = s[1] + s[2] + s[3];
}

// HBM streaming floor (tooling): mode 0 triad a = b + s c (2 reads, 1 write), 1 read-only (sum of b,
// one partial per workgroup), 2 copy a = b.  16-B accesses, 4 independent ones per lane in flight.
__global__ __launch_bounds__(BLOCK) void k_probe_stream(double* __restrict__ a, const double* __restrict__ b,
                                                       const double* __restrict__ c, double s, int64_t n2, int mode,
                                                       double* __restrict__ part) {
  constexpr int U = 4;
  const int64_t base = int64_t(blockIdx.x) * BLOCK * U + threadIdx.x;
  const d2* B = reinterpret_cast<const d2*>(b);
  const d2* C = reinterpret_cast<const d2*>(c);
  d2* A = reinterpret_cast<d2*>(a);
  d2 acc = {0.0, 0.0};
  d2 vb[U], vc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + int64_t(u) * BLOCK;
    vb[u] = i < n2 ? B[i] : d2{0.0, 0.0};
    vc[u] = (mode == 0 && i < n2) ? C[i] : d2{0.0, 0.0};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + int64_t(u) * BLOCK;
    if (mode == 1) {
      acc += vb[u];
    } else if (i < n2) {
      A[i] = mode == 0 ? vb[u] + s * vc[u] : vb[u];
    }
  }
  if (mode == 1) {
    double t = acc[0] + acc[1];
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if ((threadIdx.x & 63) == 0) part[blockIdx.x * (BLOCK / 64) + threadIdx.x / 64] = t;
  }
}

}  // namespace

// ======================================================================== C-ABI
struct gnk_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  Geo geo{0, 0, 0};
  Coef coef{};
  double* scratch = nullptr;
  double* ident = nullptr;     // 16², 32², 48², 64² identities (RinvAug of an unpreconditioned pass)
  int num_cus = 256;
  std::unordered_map<const void*, int> resident;   // kernel -> resident workgroups per CU (BLOCK threads)
  std::string err;
  // gnk_set_reduce_pairs: compensated reductions written as unevaluated (s, c) pairs
  int pairs = 0;
  // gnk_set_segments: reduction segment rows (0: off) and this slab's segment count
  int64_t seg = 0;
  int nseg = 1;
  // reductions that ran on the per-slab decomposition while segments were on (gnk_segment_fallbacks)
  int64_t seg_fallbacks = 0;
  // gnk_set_tuning (tooling A/B of kernel choices; 0 = the product's choice)
  int tune[GNK_TUNE_COUNT] = {};
  // per-launch timer (tooling, see gnk_timer_start)
  unsigned timer_mask = 0;     // bit id: kernel class id is timed
  int timer_count = 0;
  std::vector<hipEvent_t> timer_ev;
  std::vector<double> timer_bytes;
  std::vector<int> timer_ids;
};

namespace {

int fail(gnk_ctx* ctx, const std::string& msg, int code = -1) {
  if (ctx) ctx->err = msg;
  return code;
}

int check_launch(gnk_ctx* ctx, const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(ctx, std::string(what) + ": " + hipGetErrorString(e), -2);
  return 0;
}

bool ready(gnk_ctx* ctx) {
  if (!ctx) return false;
  if (ctx->geo.N <= 0) {
    ctx->err = "gnk_set_bratu has not been called";
    return false;
  }
  return true;
}

// launch geometry for local rows [lr0, lr0 + nlr), VEC elements per thread
RowLaunch rows(const gnk_ctx* ctx, int64_t lr0, int64_t nlr, int vec, int cap_blocks = MAX_RED_BLOCKS) {
  RowLaunch L;
  const int64_t per_block = int64_t(BLOCK) * vec;
  const int64_t bx = (ctx->geo.N + per_block - 1) / per_block;
  int64_t by = std::max<int64_t>(1, cap_blocks / bx);
  by = std::min<int64_t>(by, std::max<int64_t>(nlr, 1));
  by = std::min<int64_t>(by, 65535);
  L.grid = dim3(unsigned(bx), unsigned(by), 1);
  L.lr0 = lr0;
  L.nlr = nlr;
  return L;
}

// Workgroups (of `block` threads) of `fn` resident on the whole device at once: a persistent
// grid-stride launch sized to a multiple of it has no partly filled last round (at 8192^2 the trial
// kernel's former fixed 2048 workgroups were 1.6 rounds at 5 waves per SIMD).
int resident_blocks(gnk_ctx* ctx, const void* fn, int block = BLOCK, size_t lds = 0) {
  int per = 0;
  const auto it = ctx->resident.find(fn);     // (a kernel's dynamic LDS is fixed by its template arguments)
  if (it != ctx->resident.end()) {
    per = it->second;
  } else {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, block, lds) != hipSuccess || per < 1) per = 1;
    ctx->resident[fn] = per;
  }
  return per * ctx->num_cus;
}

int vec_of(const gnk_ctx* ctx) { return (ctx->geo.N % 2 == 0) ? 2 : 1; }

// ---------------------------------------------------------------- fixed reduction decompositions
// Every reduction's partial-sum decomposition is a function of the problem geometry (N, the slab's rows,
// seg_rows) and of the kernel instance only -- never of the occupancy query or the device's CU count (VERDICT r5
// #2: the persistent kernels once sized their grids from hipOccupancyMaxActiveBlocksPerMultiprocessor, so a
// register-allocation change of 130 -> 128 VGPRs re-decomposed h = V^T g and moved C2's converged-step tie).
// The grids of the persistent kernels are the tables below (workgroups per CU) times DECOMP_CUS: the occupancy
// of each instance at the round-6 build on MI355X (256 CUs), so the default grid is one full round of resident
// workgroups there.  A build whose occupancy differs runs the same grid in more (or partly filled) rounds --
// performance only; gnk_decomp_check reports table and live occupancy side by side.
constexpr int DECOMP_CUS = 256;
// k_gemv_vjpg<VEC, KCT, PEND>: [VEC - 1][PEND][KCT - 1]
constexpr unsigned char VJPG_PER_CU[2][2][24] = {
    {{8, 7, 6, 5, 5, 4, 4, 4, 4, 3, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2},
     {7, 6, 5, 4, 4, 4, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1}},
    {{7, 7, 6, 5, 5, 5, 4, 4, 4, 4, 4, 3, 3, 3, 3, 3, 3, 3, 2, 2, 2, 2, 2, 2},
     {6, 6, 5, 5, 5, 4, 4, 4, 4, 4, 3, 3, 3, 3, 2, 2, 3, 2, 2, 2, 2, 2, 2, 2}}};
constexpr int GEMVP_PER_CU = 8;                              // k_gemv_p<1>, k_gemv_p<2>
constexpr int GRAMX_PER_CU[8] = {0, 0, 2, 2, 2, 1, 1, 1};    // k_gram_x<NB> (8-wave workgroups, LDS included)
constexpr int CGM_PER_CU = 5;                                // k_cg_matvec_m<false / true>

int vjpg_decomp_blocks(int vec, bool pend, int kct) { return int(VJPG_PER_CU[vec - 1][pend ? 1 : 0][kct - 1]) * DECOMP_CUS; }

// GNK_TUNE_DECOMP_LDS: extra dynamic LDS per workgroup of the persistent kernels (tests: fewer resident workgroups,
// the same grid, so the same bits)
size_t decomp_lds(const gnk_ctx* ctx);

// k_jvp2 / k_forward2 apply (whole waves of two-point lanes, one block per row segment): turn L (a
// one-pass row launch) into their grid of row pairs; false leaves L as it was
bool rows2(const gnk_ctx* ctx, RowLaunch& L) {
  if (ctx->geo.N % ROWS2_ALIGN != 0 || L.nlr < 1) return false;
  L.grid.y = unsigned(std::min<int64_t>((L.nlr + 1) / 2, 65535));
  return true;
}

int64_t owned_lr0() { return G; }

// Segment reductions (gnk_set_segments) over one-row-per-block launches: a row launch whose partials are
// one block row per grid row (grid.y == nlr), so the partials of owned row m sit at (G - lr0 + m) * grid.x
// and a segment's rows are seg * grid.x consecutive blocks whatever the slab.  cap for rows().
int seg_row_cap(const gnk_ctx* ctx, int cap = MAX_RED_BLOCKS) { return ctx->seg > 0 ? (1 << 30) : cap; }

// Rows per range of a (range, strip) Gram grid under segments: the range count the kernel would take for a
// slab of one segment (nr_seg), rounded so that ranges tile every segment (rpr | seg) and a segment's units
// (ranges x strips) fill whole blocks of `unit` (BLOCK / 64 waves of the VALU kernels, 1 workgroup of
// the staged one).  A function of N and seg only, so every slab decomposes its segments the same way.  0: none fits.
int64_t seg_rpr(int64_t seg, int64_t nr_seg, int64_t nstrips, int64_t unit) {
  for (int64_t rpr = (seg + nr_seg - 1) / nr_seg; rpr >= 1; --rpr)
    if (seg % rpr == 0 && ((seg / rpr) * nstrips) % unit == 0) return rpr;
  return 0;
}

// local rows of the residual: owned +- 1 clipped to the domain
void residual_rows(const gnk_ctx* ctx, int64_t& lr0, int64_t& nlr) {
  const Geo& g = ctx->geo;
  int64_t lo = G - 1, hi = G + g.nrows + 1;       // [lo, hi)
  if (g.row0 == 0) lo = G;                        // global row -1 is outside
  if (g.row0 + g.nrows >= g.N) hi = G + g.nrows;  // global row N is outside
  lr0 = lo;
  nlr = hi - lo;
}

// records an event pair around one launch of the timed kernel
struct TimedLaunch {
  gnk_ctx* ctx;
  int slot = -1;
  TimedLaunch(gnk_ctx* c, int kernel_id, double bytes) : ctx(c) {
    if ((c->timer_mask >> kernel_id & 1u) && c->timer_count < int(c->timer_bytes.size())) {
      slot = c->timer_count++;
      c->timer_bytes[slot] = bytes;
      c->timer_ids[slot] = kernel_id;
      (void)hipEventRecord(c->timer_ev[2 * slot], c->stream);
    }
  }
  void done() {
    if (slot >= 0) (void)hipEventRecord(ctx->timer_ev[2 * slot + 1], ctx->stream);
    slot = -1;
  }
};

// Deterministic reduction of nblk partial blocks into out[0..len): output j reads
// partial[(j / cw) * cs + (j % cw) + b * sb].  Above 4096 partials a first stage folds
// fixed ranges of 4096 into a scratch tail, a second stage folds those.
int wreduce(gnk_ctx* ctx, const double* partial, int nblk, int len, int64_t sb, int cw, int64_t cs,
            const int* is_max, double* out) {
  constexpr int SPAN = 4096;
  if (nblk <= SPAN) {
    hipLaunchKernelGGL(k_wave_reduce, dim3(len, 1), dim3(64), 0, ctx->stream, partial, nblk, nblk, sb, cw, cs, is_max,
                       out);
    return check_launch(ctx, "reduce");
  }
  const int nsplit = (nblk + SPAN - 1) / SPAN;
  double* tmp = ctx->scratch + (SCRATCH_DOUBLES - size_t(len) * nsplit);
  hipLaunchKernelGGL(k_wave_reduce, dim3(len, nsplit), dim3(64), 0, ctx->stream, partial, nblk, SPAN, sb, cw, cs,
                     is_max, tmp);
  int rc = check_launch(ctx, "reduce stage 1");
  if (rc) return rc;
  hipLaunchKernelGGL(k_wave_reduce, dim3(len, 1), dim3(64), 0, ctx->stream, tmp, nsplit, nsplit, int64_t(1), 1,
                     int64_t(nsplit), is_max, out);
  return check_launch(ctx, "reduce stage 2");
}

int reduce(gnk_ctx* ctx, const double* partial, int nblk, int len, int stride, const int* is_max, double* out) {
  return wreduce(ctx, partial, nblk, len, stride, len, 0, is_max, out);
}

// Segment reductions (gnk_set_segments): the partials of ctx->nseg segments, segblk blocks each
// (segment s = blocks s * segblk .. (s + 1) * segblk - 1), are reduced per segment exactly as a slab of one
// segment reduces its segblk blocks (the same split and wave tree: the result depends on segblk only), then
// the segment values are folded in the fixed tree order (k_seg_fold).  The two workspaces sit below the last
// 512 Ki doubles of the arena (callers' outputs live there); partials must end before SEG_WS.
constexpr size_t SEG_WS = SCRATCH_DOUBLES - (size_t(1) << 21);
constexpr size_t SEG_WS2 = SCRATCH_DOUBLES - (size_t(1) << 20);
constexpr size_t SEG_WS_END = SCRATCH_DOUBLES - (size_t(1) << 19);
bool seg_on(const gnk_ctx* ctx) { return ctx->seg > 0; }

// Up to two reductions (b.len == 0: one) in one launch when their shapes allow it -- at most 4096 blocks
// (per segment) and at most 8 segments -- else as separate sreduce calls; the same bits either way
// (k_wave_reduce_n / k_seg_reduce_n share k_wave_reduce's per-wave arithmetic and k_seg_fold's order).
// desc.nblk: blocks per segment with segments, else all blocks.
int sreduce(gnk_ctx* ctx, const double* partial, int segblk, int len, int64_t sb, int cw, int64_t cs,
            const int* is_max, double* out);
int sreduce_n(gnk_ctx* ctx, const RedDesc& a, const RedDesc& b) {
  constexpr int SPAN = 4096;
  const bool fits = a.nblk >= 1 && a.nblk <= SPAN && (b.len == 0 || (b.nblk >= 1 && b.nblk <= SPAN));
  if (fits && a.len + b.len > 0 && !seg_on(ctx)) {
    hipLaunchKernelGGL(k_wave_reduce_n, dim3(a.len + b.len), dim3(64), 0, ctx->stream, a, b);
    return check_launch(ctx, "reduce (fused)");
  }
  if (fits && a.len + b.len > 0 && ctx->nseg <= 8) {
    hipLaunchKernelGGL(k_seg_reduce_n, dim3(a.len + b.len), dim3(512), 0, ctx->stream, a, b, ctx->nseg);
    return check_launch(ctx, "segment reduce (fused)");
  }
  int rc = sreduce(ctx, a.partial, a.nblk, a.len, a.sb, a.cw, a.cs, a.is_max, a.out);
  if (rc || b.len == 0) return rc;
  return sreduce(ctx, b.partial, b.nblk, b.len, b.sb, b.cw, b.cs, b.is_max, b.out);
}

int sreduce(gnk_ctx* ctx, const double* partial, int segblk, int len, int64_t sb, int cw, int64_t cs,
            const int* is_max, double* out) {
  if (!seg_on(ctx)) return wreduce(ctx, partial, segblk, len, sb, cw, cs, is_max, out);
  constexpr int SPAN = 4096;
  const int nseg = ctx->nseg;
  if (len > 0 && nseg <= 8 && segblk >= 1 && segblk <= SPAN) {   // one launch: the per-segment sums and their fold
    const RedDesc a{partial, segblk, sb, cw, cs, is_max, out, len}, none{partial, 1, 1, 1, 0, nullptr, out, 0};
    return sreduce_n(ctx, a, none);
  }
  const int span = std::min(SPAN, std::max(1, segblk));
  const int nsps = (std::max(1, segblk) + span - 1) / span;
  double* t1 = ctx->scratch + SEG_WS;
  double* t2 = ctx->scratch + SEG_WS2;
  if (size_t(len) * nseg * nsps > SEG_WS2 - SEG_WS || size_t(len) * nseg > SEG_WS_END - SEG_WS2)
    return fail(ctx, "segment reduction: workspace too small");
  hipLaunchKernelGGL(k_wave_reduce, dim3(len, nseg * nsps), dim3(64), 0, ctx->stream, partial, nseg * segblk, span,
                     sb, cw, cs, is_max, t1, segblk);
  int rc = check_launch(ctx, "segment reduce");
  if (rc) return rc;
  if (nsps > 1) {
    hipLaunchKernelGGL(k_wave_reduce, dim3(len, nseg), dim3(64), 0, ctx->stream, t1, nseg * nsps, nsps, int64_t(1), 1,
                       int64_t(nseg) * nsps, is_max, t2, 0);
    rc = check_launch(ctx, "segment reduce stage 2");
    if (rc) return rc;
    t1 = t2;
  }
  hipLaunchKernelGGL(k_seg_fold, dim3((len + 63) / 64), dim3(64), 0, ctx->stream, t1, nseg, len, is_max, out);
  return check_launch(ctx, "segment fold");
}

// reduce() with segments: nblk partial blocks of `stride` doubles per segment
int sreduce_rows(gnk_ctx* ctx, const double* partial, int segblk, int len, int stride, const int* is_max, double* out) {
  return sreduce(ctx, partial, segblk, len, stride, len, 0, is_max, out);
}

// Compensated reduction of nblk blocks of (s, c) pairs: quantity j of block b at
// partial[2 j + b * sb + {0, 1}] -> out[j] = s + c (k_wave_reduce2; two stages above 4096 blocks).
// With ctx->pairs the result stays the unevaluated pair: out[2 j] = s_j, out[2 j + 1] = c_j (the
// caller merges ranks' pairs, slab.Comm.sum_pairs).
int wreduce2(gnk_ctx* ctx, const double* partial, int nblk, int len, int64_t sb, double* out, int segblk = 0) {
  constexpr int SPAN = 4096;
  const int final = ctx->pairs ? 0 : 1;
  if (segblk > 0 && seg_on(ctx) && !ctx->pairs) {
    // per segment: the compensated sum of its blocks (rounded once), then the tree fold (plain)
    const int nseg = ctx->nseg;
    const int span = std::min(SPAN, segblk);
    const int nsps = (segblk + span - 1) / span;
    double* t1 = ctx->scratch + SEG_WS;
    double* t2 = ctx->scratch + SEG_WS2;
    if (size_t(2) * len * nseg * nsps > SEG_WS2 - SEG_WS || size_t(len) * nseg > SEG_WS_END - SEG_WS2)
      return fail(ctx, "segment reduction (compensated): workspace too small");
    hipLaunchKernelGGL(k_wave_reduce2, dim3(len, nseg * nsps), dim3(64), 0, ctx->stream, partial, nseg * segblk, span,
                       sb, int64_t(2), nsps > 1 ? 0 : 1, nsps > 1 ? t1 : t2, segblk);
    int rc = check_launch(ctx, "segment reduce2");
    if (rc) return rc;
    if (nsps > 1) {
      hipLaunchKernelGGL(k_wave_reduce2, dim3(len, nseg), dim3(64), 0, ctx->stream, t1, nseg * nsps, nsps, int64_t(2),
                         int64_t(2) * nseg * nsps, 1, t2, 0);
      rc = check_launch(ctx, "segment reduce2 stage 2");
      if (rc) return rc;
    }
    hipLaunchKernelGGL(k_seg_fold, dim3((len + 63) / 64), dim3(64), 0, ctx->stream, t2, nseg, len, nullptr, out);
    return check_launch(ctx, "segment fold (compensated)");
  }
  if (segblk > 0 && seg_on(ctx)) nblk = segblk * ctx->nseg;     // pairs: every block, one rank-level pair
  if (nblk <= SPAN) {
    hipLaunchKernelGGL(k_wave_reduce2, dim3(len, 1), dim3(64), 0, ctx->stream, partial, nblk, nblk, sb, int64_t(2),
                       final, out);
    return check_launch(ctx, "reduce2");
  }
  const int nsplit = (nblk + SPAN - 1) / SPAN;
  double* tmp = ctx->scratch + (SCRATCH_DOUBLES - size_t(2) * len * nsplit);
  hipLaunchKernelGGL(k_wave_reduce2, dim3(len, nsplit), dim3(64), 0, ctx->stream, partial, nblk, SPAN, sb, int64_t(2),
                     0, tmp);
  int rc = check_launch(ctx, "reduce2 stage 1");
  if (rc) return rc;
  hipLaunchKernelGGL(k_wave_reduce2, dim3(len, 1), dim3(64), 0, ctx->stream, tmp, nsplit, nsplit, int64_t(2),
                     int64_t(2) * nsplit, final, out);
  return check_launch(ctx, "reduce2 stage 2");
}

// device constant {0, 1} flags for {sum, max} reductions
__device__ int d_sum_max_flags[2] = {0, 1};

const int* sum_max_flags() {
  void* p = nullptr;
  (void)hipGetSymbolAddress(&p, HIP_SYMBOL(d_sum_max_flags));
  return static_cast<const int*>(p);
}

// {sum x^2, max |x|} of k_stats partials ([s, c, max] per block); ctx->pairs: {s, c, max |x|}.
// Segments: nblk blocks per segment.
int reduce_stats(gnk_ctx* ctx, const double* partial, int nblk, double* stats_out) {
  const bool sg = seg_on(ctx);
  int rc = wreduce2(ctx, partial, nblk, 1, 3, stats_out, sg ? nblk : 0);
  if (rc) return rc;
  return sreduce(ctx, partial + 2, nblk, 1, 3, 1, 0, sum_max_flags() + 1, stats_out + (ctx->pairs ? 2 : 1));
}

int tuning(const gnk_ctx* ctx, int key) { return ctx->tune[key]; }

size_t decomp_lds(const gnk_ctx* ctx) { return size_t(std::max(0, std::min(ctx->tune[GNK_TUNE_DECOMP_LDS], 96 * 1024))); }

// flat geometry helpers (generic problems)
bool ctx_ok(gnk_ctx* ctx) { return ctx != nullptr; }
int flat_vec(int64_t n, int64_t ldv = 0) { return (n % 2 == 0 && ldv % 2 == 0) ? 2 : 1; }
// the two-point paths of the streaming kernels move 16-B pairs: a flat vector that is not 16-B aligned (a view
// at an odd offset; NULL counts as aligned) runs one point per lane
bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
RowLaunch flat_rows(int64_t n, int vec, int cap = MAX_RED_BLOCKS) {
  RowLaunch L;
  const int64_t per = int64_t(BLOCK) * vec;
  const int64_t bx = std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, cap));
  L.grid = dim3(unsigned(bx), 1, 1);
  L.lr0 = 0;
  L.nlr = 1;
  return L;
}

}  // namespace

extern "C" {

int gnk_abi_version(void) { return GNK_ABI_VERSION; }

int64_t gnk_segment_fallbacks(const gnk_ctx* ctx) { return ctx ? ctx->seg_fallbacks : -1; }

int gnk_ctx_create(int device, gnk_ctx** out) {
  if (!out) return -1;
  *out = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return -2;
  auto* ctx = new gnk_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->num_cus = prop.multiProcessorCount;
  e = hipMalloc(&ctx->scratch, SCRATCH_DOUBLES * sizeof(double));
  if (e != hipSuccess) {
    delete ctx;
    return -3;
  }
  {
    std::vector<double> id(ident_offset(5), 0.0);
    for (int b = 1; b <= 4; ++b)
      for (int i = 0; i < 16 * b; ++i) id[ident_offset(b) + i * 16 * b + i] = 1.0;
    e = hipMalloc(&ctx->ident, id.size() * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(ctx->ident, id.data(), id.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(ctx->scratch);
      delete ctx;
      return -3;
    }
  }
  *out = ctx;
  return 0;
}

void gnk_ctx_destroy(gnk_ctx* ctx) {
  if (!ctx) return;
  for (hipEvent_t e : ctx->timer_ev) (void)hipEventDestroy(e);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->ident) (void)hipFree(ctx->ident);
  delete ctx;
}

const char* gnk_last_error(const gnk_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int gnk_set_reduce_pairs(gnk_ctx* ctx, int on) {
  if (!ctx) return -1;
  ctx->pairs = on ? 1 : 0;
  return 0;
}

int gnk_set_tuning(gnk_ctx* ctx, int key, int value) {
  if (!ctx) return -1;
  if (key < 0 || key >= GNK_TUNE_COUNT) return fail(ctx, "gnk_set_tuning: unknown key");
  ctx->tune[key] = value;
  return 0;
}

int64_t gnk_scratch_doubles(void) { return int64_t(SCRATCH_DOUBLES); }

int gnk_set_stream(gnk_ctx* ctx, void* stream) {
  if (!ctx) return -1;
  ctx->stream = static_cast<hipStream_t>(stream);
  return 0;
}

int gnk_set_bratu(gnk_ctx* ctx, int64_t N, int64_t row0, int64_t nrows, double h, double alpha, double lambda) {
  if (!ctx) return -1;
  if (N < 2 || nrows < 1 || row0 < 0 || row0 + nrows > N) return fail(ctx, "gnk_set_bratu: bad slab geometry");
  if (nrows < G && nrows != N) return fail(ctx, "gnk_set_bratu: slab must own >= GNK_GHOST_ROWS rows");
  ctx->geo = Geo{N, row0, nrows};
  ctx->seg = 0;                                     // segments belong to one slab geometry
  ctx->nseg = 1;
  Coef c;
  // identical float expressions to ref:bratu_pde_problem.py:58,67 (h ** -2, h ** -1)
  const double hm2 = std::pow(h, -2.0);
  const double hm1 = std::pow(h, -1.0);
  c.hm2 = -(-1.0 * hm2);
  c.l_off = -1.0 * hm2;
  c.l_diag = 4.0 * hm2;
  c.dx_diag = alpha * (-1.0 * hm1);
  c.dx_up = alpha * (1.0 * hm1);
  c.j_lin_diag = c.l_diag + c.dx_diag;
  c.j_lin_up = c.l_off + c.dx_up;
  c.lam = lambda;
  c.lam_zero = (lambda == 0.0) ? 1 : 0;
  ctx->coef = c;
  return 0;
}

int gnk_set_segments(gnk_ctx* ctx, int64_t seg_rows) {
  if (!ready(ctx)) return -1;
  if (seg_rows == 0) {
    ctx->seg = 0;
    ctx->nseg = 1;
    return 0;
  }
  const Geo& g = ctx->geo;
  if (seg_rows < 1 || g.row0 % seg_rows != 0 || g.nrows % seg_rows != 0)
    return fail(ctx, "gnk_set_segments: the slab must hold whole segments (row0 % seg_rows == nrows % seg_rows == 0)");
  if (g.nrows / seg_rows > SEG_MAX) return fail(ctx, "gnk_set_segments: more than 64 segments per slab");
  if (g.nrows > 65535) return fail(ctx, "gnk_set_segments: more than 65535 rows per slab");
  ctx->seg = seg_rows;
  ctx->nseg = int(g.nrows / seg_rows);
  return 0;
}

int64_t gnk_slab_len(const gnk_ctx* ctx) {
  if (!ctx) return -1;
  return (ctx->geo.nrows + 2 * G) * ctx->geo.N;
}

#define DISPATCH_VEC(ctx, KERNEL, L, SHMEM, ...)                                                     \
  do {                                                                                              \
    if (vec_of(ctx) == 2)                                                                           \
      hipLaunchKernelGGL(KERNEL<2>, L.grid, dim3(BLOCK), SHMEM, ctx->stream, __VA_ARGS__);          \
    else                                                                                            \
      hipLaunchKernelGGL(KERNEL<1>, L.grid, dim3(BLOCK), SHMEM, ctx->stream, __VA_ARGS__);          \
  } while (0)

int gnk_bratu_jvp(gnk_ctx* ctx, const double* u, const double* v, double* out) {
  if (!ready(ctx)) return -1;
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);
  TimedLaunch tl(ctx, GNK_TIMER_JVP, 24.0 * double(ctx->geo.nrows) * double(ctx->geo.N));
  if (rows2(ctx, L))
    hipLaunchKernelGGL(k_jvp2<false>, L.grid, dim3(BLOCK), 0, ctx->stream, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr);
  else
    DISPATCH_VEC(ctx, k_jvp, L, 0, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr, 0);
  tl.done();
  return check_launch(ctx, "bratu_jvp");
}

int gnk_bratu_vjp(gnk_ctx* ctx, const double* u, const double* w, double* out) {
  if (!ready(ctx)) return -1;
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);
  if (rows2(ctx, L))
    hipLaunchKernelGGL(k_jvp2<true>, L.grid, dim3(BLOCK), 0, ctx->stream, u, w, out, ctx->geo, ctx->coef, L.lr0, L.nlr);
  else
    DISPATCH_VEC(ctx, k_jvp, L, 0, u, w, out, ctx->geo, ctx->coef, L.lr0, L.nlr, 1);
  return check_launch(ctx, "bratu_vjp");
}

int gnk_bratu_forward(gnk_ctx* ctx, const double* x, double* F) {
  if (!ready(ctx)) return -1;
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);
  if (rows2(ctx, L))
    hipLaunchKernelGGL(k_forward2, L.grid, dim3(BLOCK), 0, ctx->stream, x, (const double*)nullptr, F, ctx->geo,
                       ctx->coef, L.lr0, L.nlr, (double*)nullptr);
  else
    DISPATCH_VEC(ctx, k_forward, L, 0, x, (const double*)nullptr, F, ctx->geo, ctx->coef, L.lr0, L.nlr,
                 (double*)nullptr);
  return check_launch(ctx, "bratu_forward");
}

int gnk_bratu_residual(gnk_ctx* ctx, const double* x, const double* y, double* r, double* norm2_out) {
  if (!ready(ctx)) return -1;
  if (!y) return fail(ctx, "bratu_residual: y is NULL");
  int64_t lr0, nlr;
  residual_rows(ctx, lr0, nlr);
  // one workgroup per row chunk (a persistent grid of the resident workgroups measured 17 % slower:
  // 0.37 vs 0.32 ms at 8192^2, profiles/round3/rocprof_window_breakdown.json)
  RowLaunch L = rows(ctx, lr0, nlr, vec_of(ctx), seg_row_cap(ctx));
  const int nblk = L.grid.x * L.grid.y;
  if (seg_on(ctx) && int64_t(L.grid.y) != L.nlr) return fail(ctx, "bratu_residual: segments need one block row per grid row");
  // two rows per block where k_forward runs one row per block (its partials, bit for bit)
  if (int64_t(L.grid.y) == L.nlr && rows2(ctx, L))
    hipLaunchKernelGGL(k_forward2, L.grid, dim3(BLOCK), 0, ctx->stream, x, y, r, ctx->geo, ctx->coef, L.lr0, L.nlr,
                       ctx->scratch);
  else
    DISPATCH_VEC(ctx, k_forward, L, 0, x, y, r, ctx->geo, ctx->coef, L.lr0, L.nlr, ctx->scratch);
  int rc = check_launch(ctx, "bratu_residual");
  if (rc) return rc;
  if (norm2_out && seg_on(ctx))     // owned row m's partials at (G - lr0 + m) * grid.x
    return sreduce_rows(ctx, ctx->scratch + (G - L.lr0) * L.grid.x, int(ctx->seg * L.grid.x), 1, 1, nullptr, norm2_out);
  if (norm2_out) return reduce(ctx, ctx->scratch, nblk, 1, 1, nullptr, norm2_out);
  return 0;
}

int gnk_bratu_diag_jtj(gnk_ctx* ctx, const double* u, double* out, int reciprocal) {
  if (!ready(ctx)) return -1;
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);
  DISPATCH_VEC(ctx, k_diag_jtj, L, 0, u, out, ctx->geo, ctx->coef, L.lr0, L.nlr, reciprocal);
  return check_launch(ctx, "bratu_diag_jtj");
}

int gnk_bratu_jdiag(gnk_ctx* ctx, const double* u, double* d) {
  if (!ready(ctx)) return -1;
  int64_t lr0, nlr;
  residual_rows(ctx, lr0, nlr);
  RowLaunch L = rows(ctx, lr0, nlr, vec_of(ctx), 1 << 30);
  DISPATCH_VEC(ctx, k_jdiag, L, 0, u, d, ctx->geo, ctx->coef, L.lr0, L.nlr);
  return check_launch(ctx, "bratu_jdiag");
}

int gnk_basis_gemv(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c, double* x) {
  if (!ready(ctx)) return -1;
  if (k < 1) return fail(ctx, "basis_gemv: k < 1");
  if (vec_of(ctx) == 2 && (ldv % 2 != 0)) return fail(ctx, "basis_gemv: ldv must be even");
  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), 1 << 30);
  DISPATCH_VEC(ctx, k_gemv, L, 0, V, ldv, k, c, x, ctx->geo, L.lr0, L.nlr);
  return check_launch(ctx, "basis_gemv");
}

int gnk_vjp_gemv_t(gnk_ctx* ctx, const double* u, const double* r, const double* V, int64_t ldv, int k,
                   double* g, double* h_out) {
  if (!ready(ctx)) return -1;
  if (k < 0) return fail(ctx, "vjp_gemv_t: k < 0");
  if (k > 0 && !V) return fail(ctx, "vjp_gemv_t: V is NULL");
  if (vec_of(ctx) == 2 && (ldv % 2 != 0)) return fail(ctx, "vjp_gemv_t: ldv must be even");
  // one chunk of the smallest compiled width >= k up to 24 columns, else 16-column chunks
  const int kct = k <= 24 ? std::max(4, (k + 3) / 4 * 4) : 16;
  const int nchunk = std::max(1, (k + kct - 1) / kct);
  const int cap = tuning(ctx, GNK_TUNE_VJPG_BLOCKS);
  // blocks per chunk: ~2048 in all, at least 512 per chunk (the first chunk, which computes g, runs alone in
  // the wide split below: at 2048 / 7 = 292 it kept ~1 workgroup per CU)
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx),
                     seg_on(ctx) ? (1 << 30) : (cap > 0 ? cap : std::max(512, 2048 / nchunk)));
  const int nblk = L.grid.x * L.grid.y;
  // column chunks per launch: with segments every owned row has its own block row (nblk = grid.x * rows), and
  // a wide basis (C5: k up to 200) on a large slab would overflow the partials' workspace -- then the chunks
  // go in several launches (each chunk's arithmetic and reduction unchanged; only the launch containing
  // chunk 0 stores g)
  const size_t room = SEG_WS;
  if (size_t(nblk) * kct > room) return fail(ctx, "vjp_gemv_t: scratch too small");
  const int zt = tuning(ctx, GNK_TUNE_VJPG_ZMAX);
  const int zmax = int(std::min<size_t>(std::min<size_t>(size_t(nchunk), room / (size_t(nblk) * kct)),
                                        zt > 0 ? size_t(zt) : size_t(nchunk)));
  // several 16-column chunks: chunk 0 computes and stores g, the rest read it back in 32-column chunks
  // (each chunk recomputing g from u and r re-read 4 grid vectors: 28 of 128 at k = 100), on the same
  // row decomposition -- every column's partials, and so h, bit for bit those of the one-launch form
  if (nchunk > 1 && zt == 0 && g && vec_of(ctx) == 2 && size_t(nblk) * 32 <= room) {
    L.grid.z = 1;
    hipLaunchKernelGGL((k_vjp_gemv_t<2, 16>), L.grid, dim3(BLOCK), 0, ctx->stream, u, r, V, ldv, std::min(k, 16), g,
                       ctx->geo, ctx->coef, L.lr0, L.nlr, ctx->scratch, 0);
    int rc = check_launch(ctx, "vjp_gemv_t (chunk 0)");
    if (rc) return rc;
    if (h_out) {
      rc = seg_on(ctx) ? sreduce(ctx, ctx->scratch, int(ctx->seg * L.grid.x), 16, 16, 16, int64_t(nblk) * 16, nullptr,
                                 h_out)
                       : wreduce(ctx, ctx->scratch, nblk, 16, 16, 16, int64_t(nblk) * 16, nullptr, h_out);
      if (rc) return rc;
    }
    const int kr = k - 16, nc32 = (kr + 31) / 32;
    const int zm = int(std::min<size_t>(size_t(nc32), room / (size_t(nblk) * 32)));
    for (int z0 = 0; z0 < nc32; z0 += zm) {
      const int nz = std::min(zm, nc32 - z0);
      L.grid.z = unsigned(nz);
      hipLaunchKernelGGL((k_vjp_gemv_t<2, 32, true>), L.grid, dim3(BLOCK), 0, ctx->stream, u, r, V + 16 * ldv, ldv, kr,
                         g, ctx->geo, ctx->coef, L.lr0, L.nlr, ctx->scratch, z0);
      rc = check_launch(ctx, "vjp_gemv_t (read g)");
      if (rc) return rc;
      if (!h_out) continue;
      const int len = std::min(kr - z0 * 32, nz * 32);
      double* ho = h_out + 16 + int64_t(z0) * 32;
      rc = seg_on(ctx) ? sreduce(ctx, ctx->scratch, int(ctx->seg * L.grid.x), len, 32, 32, int64_t(nblk) * 32, nullptr,
                                 ho)
                       : wreduce(ctx, ctx->scratch, nblk, len, 32, 32, int64_t(nblk) * 32, nullptr, ho);
      if (rc) return rc;
    }
    return 0;
  }
  for (int z0 = 0; z0 < nchunk; z0 += zmax) {
    const int nz = std::min(zmax, nchunk - z0);
    L.grid.z = unsigned(nz);
#define VJPG_LAUNCH(V_, K_)                                                                                 \
  hipLaunchKernelGGL((k_vjp_gemv_t<V_, K_>), L.grid, dim3(BLOCK), 0, ctx->stream, u, r, V, ldv, k, g, ctx->geo, \
                     ctx->coef, L.lr0, L.nlr, ctx->scratch, z0)
#define VJPG_SWITCH(V_)                  \
  switch (kct) {                         \
    case 4: VJPG_LAUNCH(V_, 4); break;   \
    case 8: VJPG_LAUNCH(V_, 8); break;   \
    case 12: VJPG_LAUNCH(V_, 12); break; \
    case 16: VJPG_LAUNCH(V_, 16); break; \
    case 20: VJPG_LAUNCH(V_, 20); break; \
    default: VJPG_LAUNCH(V_, 24); break; \
  }
    if (vec_of(ctx) == 2) {
      VJPG_SWITCH(2)
    } else {
      VJPG_SWITCH(1)
    }
#undef VJPG_SWITCH
#undef VJPG_LAUNCH
    int rc = check_launch(ctx, "vjp_gemv_t");
    if (rc) return rc;
    if (k == 0 || !h_out) continue;
    const int len = std::min(k - z0 * kct, nz * kct);
    if (seg_on(ctx))                // one block row per owned row: segment s = blocks s * seg * grid.x ..
      rc = sreduce(ctx, ctx->scratch, int(ctx->seg * L.grid.x), len, kct, kct, int64_t(nblk) * kct, nullptr,
                   h_out + int64_t(z0) * kct);
    else
      rc = wreduce(ctx, ctx->scratch, nblk, len, kct, kct, int64_t(nblk) * kct, nullptr, h_out + int64_t(z0) * kct);
    if (rc) return rc;
  }
  return 0;
}

}  // extern "C"
namespace {
// k_gemv_vjpg<VEC, kct, PEND> for kct = 1 .. 24
template <int V_, bool P_, int... K>
const void* vjpg_table(int kct, std::integer_sequence<int, K...>) {
  static const void* const t[] = {reinterpret_cast<const void*>(&k_gemv_vjpg<V_, K + 1, P_>)...};
  return t[kct - 1];
}
template <int V_, bool P_>
const void* vjpg_pick(int kct) { return vjpg_table<V_, P_>(kct, std::make_integer_sequence<int, 24>{}); }
}  // namespace
extern "C" {

// The wide fused first trial (k_trial_w, 25..208 columns) per width class (64-point tiles; ROUNDS 4 / 7 / 13 / 26:
// up to 32 / 56 / 104 / 208 columns): tiles in flight per workgroup (DEPTH), a fixed grid of TW_PER_CU workgroups
// per CU -- the decomposition of its h partials -- capped by the tiles, and the register budget that lets that
// many be resident (amdgpu_waves_per_eu: one wave per SIMD per workgroup).  8192^2, ms per launch
// (profiles/round6/trial_w_ab.jsonl): 25..32 columns depth 2 x 3 per CU 3.87-4.37 vs depth 1 x 4 4.45-5.15;
// 40..56 depth 1 x 3 5.08-6.27 vs depth 2 x 3 7.7-9.3; 64..100 depth 2 x 2 7.9-11.5 vs 2 x 3 10.2-13.2.
constexpr int TW_DEPTH[4] = {2, 1, 2, 1};
constexpr int TW_PER_CU[4] = {3, 3, 2, 1};

static int trial_w_launch(gnk_ctx* ctx, const char* what, const double* V, int64_t ldv, int k, const double* c,
                          const double* hh, const double* r, double* x, double* g, double* h_out, double* stats_out) {
  const bool pend = hh != nullptr;
  const int kk = k + (pend ? 1 : 0);
  if (kk > TW_KMAX || seg_on(ctx) || ctx->geo.N % 128 != 0 || ldv % 2 != 0)
    return fail(ctx, std::string(what) + ": more than 24 columns need N % 128 == 0, even ldv, no segments, <= 208");
  double* wcol = pend ? const_cast<double*>(V) + int64_t(k) * ldv : nullptr;
  if (pend && (g == wcol || x == wcol)) return fail(ctx, std::string(what) + ": g / x alias the pending column");
  const int cls = kk <= 32 ? 0 : kk <= 56 ? 1 : kk <= 104 ? 2 : 3;
  constexpr int TP = 64;
  // GNK_TUNE_TRIALW (tooling A/B): 16 * depth + workgroups per CU
  const int tt = tuning(ctx, GNK_TUNE_TRIALW);
  const int depth = (tt >> 4) == 1 ? 1 : (tt >> 4) == 2 ? 2 : TW_DEPTH[cls];
  const int per_cu = (tt & 15) ? (tt & 15) : TW_PER_CU[cls];
  if (cls == 3 && depth == 2) return fail(ctx, std::string(what) + ": depth 2 not built for > 104 columns");
  const int64_t ntiles = (ctx->geo.nrows + 2 * G) * (ctx->geo.N / TP);
  const int nblk = int(std::max<int64_t>(1, std::min<int64_t>(ntiles, int64_t(per_cu) * DECOMP_CUS)));
  const size_t soff = (size_t(nblk) * kk + 1) & ~size_t(1);
  if (soff + 2 * size_t(nblk) > SCRATCH_DOUBLES / 2) return fail(ctx, std::string(what) + ": scratch too small");
  double* spart = ctx->scratch + soff;
  const size_t lds = (size_t(kk) * (TP + 2) + 9 * size_t(TP) + 2 * size_t(kk)) * sizeof(double) + decomp_lds(ctx);
  if (lds > 160 * 1024) return fail(ctx, std::string(what) + ": LDS tile too large");
  TimedLaunch tl(ctx, GNK_TIMER_TRIAL, 8.0 * double(ctx->geo.nrows) * double(ctx->geo.N) * double(k + 3 + (pend ? 2 : 0)));
#define TRIALW(TV, RV, DV, PV, WV)                                                                                  \
  hipLaunchKernelGGL((k_trial_w<TV, RV, DV, PV, WV>), dim3(unsigned(nblk)), dim3(BLOCK), lds, ctx->stream, V, ldv, k, c, \
                     hh, wcol, r, x, g, ctx->geo, ctx->coef, ntiles, ctx->scratch, spart)
#define TRIALWD(TV, RV, PV, WV, WV2) do { if (depth == 2) TRIALW(TV, RV, 2, PV, WV2); else TRIALW(TV, RV, 1, PV, WV); } \
  while (0)
  // register budget (amdgpu_waves_per_eu) of each class: its workgroups per CU, one wave per SIMD each (depth 2:
  // one fewer for the two tiles' VGPRs; 2 = the default for 57..104 columns, A/B in profiles/round6/trial_w_ab.jsonl)
  if (pend) {
    if (cls == 0) TRIALWD(64, 4, true, 4, 3); else if (cls == 1) TRIALWD(64, 7, true, 3, 2);
    else if (cls == 2) TRIALWD(64, 13, true, 2, 2); else TRIALW(64, 26, 1, true, 1);
  } else {
    if (cls == 0) TRIALWD(64, 4, false, 4, 3); else if (cls == 1) TRIALWD(64, 7, false, 3, 2);
    else if (cls == 2) TRIALWD(64, 13, false, 2, 2); else TRIALW(64, 26, 1, false, 1);
  }
#undef TRIALWD
#undef TRIALW
  tl.done();
  int rc = check_launch(ctx, what);
  if (rc) return rc;
  const RedDesc dh{ctx->scratch, nblk, kk, kk, int64_t(nblk) * kk, nullptr, h_out, kk};
  const RedDesc ds{spart, nblk, 2, 2, 0, sum_max_flags(), stats_out, pend ? 2 : 0};
  return sreduce_n(ctx, dh, ds);
}

// shared body of gnk_basis_gemv_vjp_gemv_t (hh == nullptr) and its pending-column form
static int gemv_vjpg_launch(gnk_ctx* ctx, const char* what, const double* V, int64_t ldv, int k, const double* c,
                     const double* hh, const double* r, double* x, double* g, double* h_out, double* stats_out) {
  const bool pend = hh != nullptr;
  const int kk = k + (pend ? 1 : 0);
  if (k >= 1 && kk > 24 && V && c && r && x && g && h_out && (!pend || stats_out))
    return trial_w_launch(ctx, what, V, ldv, k, c, hh, r, x, g, h_out, stats_out);
  if (k < 1 || kk > 24) return fail(ctx, std::string(what) + ": columns must be in [1, 24]");
  if (!V || !c || !r || !x || !g || !h_out || (pend && !stats_out)) return fail(ctx, std::string(what) + ": NULL argument");
  if (vec_of(ctx) == 2 && (ldv % 2 != 0)) return fail(ctx, std::string(what) + ": ldv must be even");
  double* wcol = pend ? const_cast<double*>(V) + int64_t(k) * ldv : nullptr;
  if (pend && (g == wcol || x == wcol)) return fail(ctx, std::string(what) + ": g / x alias the pending column");
  // one instance per width (no clamped surplus loads), grid = one full round of resident workgroups
  const int kct = kk;
  const void* fn = vec_of(ctx) == 2 ? (pend ? vjpg_pick<2, true>(kct) : vjpg_pick<2, false>(kct))
                                    : (pend ? vjpg_pick<1, true>(kct) : vjpg_pick<1, false>(kct));
  const int dblk = vjpg_decomp_blocks(vec_of(ctx), pend, kct);     // the fixed grid (one round on MI355X)
  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), dblk);
  // segments: that grid once per segment (grid.z = nseg + 1: the segments, then the ghost rows);
  // a segment's partials then depend on the kernel instance only, not on the slab
  const int ns = seg_on(ctx) ? ctx->nseg + 1 : 1;                  // partial sets
  L.grid.z = unsigned(ns);
  if (seg_on(ctx)) L.grid.y = unsigned(std::min<int64_t>(dblk / L.grid.x, ctx->seg));
  const int nblk = L.grid.x * L.grid.y;
  const size_t soff = (size_t(nblk) * ns * kct + 1) & ~size_t(1);  // stats partials after the h partials
  if (soff + 2 * size_t(nblk) * ns > SCRATCH_DOUBLES / 2) return fail(ctx, std::string(what) + ": scratch too small");
  double* spart = ctx->scratch + soff;
  Geo geo = ctx->geo;
  Coef coef = ctx->coef;
  double* part = ctx->scratch;
  int64_t seg = ctx->seg;
  int nseg = ctx->nseg;
  void* args[] = {&V, &ldv, &k, &c, &hh, &wcol, &r, &x, &g, &geo, &coef, &L.lr0, &L.nlr, &part, &spart, &seg, &nseg};
  // algorithmic bytes (owned rows): the k settled columns, r in, x and g out; pending: w read + written
  TimedLaunch tl(ctx, GNK_TIMER_TRIAL, 8.0 * double(ctx->geo.nrows) * double(ctx->geo.N) * double(k + 3 + (pend ? 2 : 0)));
  (void)hipLaunchKernel(fn, L.grid, dim3(BLOCK), args, decomp_lds(ctx), ctx->stream);
  tl.done();
  int rc = check_launch(ctx, what);
  if (rc) return rc;
  // the h partials and (pending) the {sum w^2, max |w|} partials: one launch
  const RedDesc dh{ctx->scratch, nblk, kct, kct, int64_t(nblk) * kct, nullptr, h_out, kk};
  const RedDesc ds{spart, nblk, 2, 2, 0, sum_max_flags(), stats_out, pend ? 2 : 0};
  return sreduce_n(ctx, dh, ds);
}

int gnk_basis_gemv_vjp_gemv_t(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c, const double* r,
                              double* x, double* g, double* h_out) {
  if (!ready(ctx)) return -1;
  return gemv_vjpg_launch(ctx, "basis_gemv_vjp_gemv_t", V, ldv, k, c, nullptr, r, x, g, h_out, nullptr);
}

int gnk_basis_gemv_vjp_gemv_t_pending(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c,
                                      const double* hh, const double* r, double* x, double* g, double* h_out,
                                      double* stats_out) {
  if (!ready(ctx)) return -1;
  if (!hh) return fail(ctx, "basis_gemv_vjp_gemv_t_pending: hh is NULL");
  return gemv_vjpg_launch(ctx, "basis_gemv_vjp_gemv_t_pending", V, ldv, k, c, hh, r, x, g, h_out, stats_out);
}

int gnk_basis_gemv_pending(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c, const double* hh,
                           double* x, double* stats_out) {
  if (!ready(ctx)) return -1;
  if (k < 1) return fail(ctx, "basis_gemv_pending: k < 1");
  if (!V || !c || !hh || !x || !stats_out) return fail(ctx, "basis_gemv_pending: NULL argument");
  if (vec_of(ctx) == 2 && (ldv % 2 != 0)) return fail(ctx, "basis_gemv_pending: ldv must be even");
  double* w = const_cast<double*>(V) + int64_t(k) * ldv;
  if (x == w) return fail(ctx, "basis_gemv_pending: x aliases the pending column");
  const int dblk = GEMVP_PER_CU * DECOMP_CUS;
  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), dblk);
  if (seg_on(ctx)) {                                      // as gemv_vjpg_launch
    L.grid.z = unsigned(ctx->nseg + 1);
    L.grid.y = unsigned(std::min<int64_t>(dblk / L.grid.x, ctx->seg));
  }
  const int nblk = L.grid.x * L.grid.y;
  DISPATCH_VEC(ctx, k_gemv_p, L, decomp_lds(ctx), V, ldv, k, c, hh, w, x, ctx->geo, L.lr0, L.nlr, ctx->scratch,
               ctx->seg, ctx->nseg);
  int rc = check_launch(ctx, "basis_gemv_pending");
  if (rc) return rc;
  return sreduce_rows(ctx, ctx->scratch, nblk, 2, 2, sum_max_flags(), stats_out);
}

int gnk_cgs_update(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* h, double* g,
                   double* stats_out) {
  if (!ready(ctx)) return -1;
  if (k < 1) return fail(ctx, "cgs_update: k < 1");
  if (vec_of(ctx) == 2 && (ldv % 2 != 0)) return fail(ctx, "cgs_update: ldv must be even");
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), seg_row_cap(ctx));
  const int nblk = L.grid.x * L.grid.y;
  DISPATCH_VEC(ctx, k_cgs, L, 0, V, ldv, k, h, g, ctx->geo, L.lr0, L.nlr, ctx->scratch);
  int rc = check_launch(ctx, "cgs_update");
  if (rc) return rc;
  if (seg_on(ctx)) return sreduce_rows(ctx, ctx->scratch, int(ctx->seg * L.grid.x), 2, 2, sum_max_flags(), stats_out);
  return reduce(ctx, ctx->scratch, nblk, 2, 2, sum_max_flags(), stats_out);
}

int gnk_vec_stats(gnk_ctx* ctx, const double* x, double* stats_out) {
  if (!ready(ctx)) return -1;
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), seg_row_cap(ctx));
  const int nblk = L.grid.x * L.grid.y;
  DISPATCH_VEC(ctx, k_stats, L, 0, x, ctx->geo, L.lr0, L.nlr, ctx->scratch);
  int rc = check_launch(ctx, "vec_stats");
  if (rc) return rc;
  return reduce_stats(ctx, ctx->scratch, seg_on(ctx) ? int(ctx->seg * L.grid.x) : nblk, stats_out);
}

int gnk_vec_div(gnk_ctx* ctx, const double* src, double denom, double* dst, int full_slab) {
  if (!ready(ctx)) return -1;
  RowLaunch L = full_slab ? rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), 1 << 30)
                          : rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);
  DISPATCH_VEC(ctx, k_div, L, 0, src, denom, dst, ctx->geo, L.lr0, L.nlr);
  return check_launch(ctx, "vec_div");
}

int gnk_normalize_jnorm(gnk_ctx* ctx, const double* u, const double* g, double denom, double* v,
                        double* jnorm2_out) {
  if (!ready(ctx)) return -1;
  if (!u || !g || !v) return fail(ctx, "normalize_jnorm: NULL vector");
  if (g == v) return fail(ctx, "normalize_jnorm: v must not alias g (stencil reads of g)");
  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), seg_row_cap(ctx));
  const int nblk = L.grid.x * L.grid.y;
  // the segmented reduction below reads one block row per grid row (partials at G * grid.x, seg * grid.x);
  // rows() caps grid.y at 65535 (nrows + 2 G past that would misplace the offsets silently)
  if (seg_on(ctx) && jnorm2_out && int64_t(L.grid.y) != L.nlr)
    return fail(ctx, "normalize_jnorm: segments need one block row per grid row");
  DISPATCH_VEC(ctx, k_div_jnorm, L, 0, u, g, denom, v, ctx->geo, ctx->coef, L.lr0, L.nlr, ctx->scratch);
  int rc = check_launch(ctx, "normalize_jnorm");
  if (rc || !jnorm2_out) return rc;
  if (seg_on(ctx))                  // owned rows from grid row G
    return sreduce_rows(ctx, ctx->scratch + G * L.grid.x, int(ctx->seg * L.grid.x), 1, 1, nullptr, jnorm2_out);
  return reduce(ctx, ctx->scratch, nblk, 1, 1, nullptr, jnorm2_out);   // sum (J g)^2
}

int gnk_vec_axpy(gnk_ctx* ctx, const double* x, double alpha, const double* d, double* out, int full_slab) {
  if (!ready(ctx)) return -1;
  RowLaunch L = full_slab ? rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), 1 << 30)
                          : rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);
  DISPATCH_VEC(ctx, k_axpy, L, 0, x, alpha, d, out, ctx->geo, L.lr0, L.nlr);
  return check_launch(ctx, "vec_axpy");
}

int gnk_gram_padded_dim(int k, int with_r) { return ((k + (with_r ? 1 : 0) + 15) / 16) * 16; }

int gnk_gram(gnk_ctx* ctx, const double* u, const double* V, int64_t ldv, int k, const double* rinv, int64_t ldr,
             const double* r, double* G_out) {
  if (!ready(ctx)) return -1;
  if (k < 1) return fail(ctx, "gram: k < 1");
  const int KP = gnk_gram_padded_dim(k, r != nullptr);
  if (rinv && ldr != KP) return fail(ctx, "gram: rinv must be the kp x kp augmented inverse (ldr == kp)");
  const int nb = KP / 16;
  const int P = nb * (nb + 1) / 2;
  // VALU pass for small k with r (every preconditioned pass at k <= 9); tuning GNK_TUNE_GRAM_PATH
  // 3 disables it, 1 (tests) forces the staged kernel instead
  const int path = tuning(ctx, GNK_TUNE_GRAM_PATH);
  const int v1t = tuning(ctx, GNK_TUNE_GRAM_V1MIN);          // tooling A/B: first k of the one-point form
  int gv_kmax = v1t < 0 ? GV1_KMIN - 1 : GV_KMAX;
  // preconditioned passes: from GQ_KMIN the 4x4x4-block staged pass (k_gram_q) beats the one-point VALU kernel
  // (k = 8 / 9: 1.06 / 1.22-1.25 vs 1.19 / 1.32 ms, profiles/round6/gram_q_small_ab.jsonl)
  const int q_t = tuning(ctx, GNK_TUNE_GRAM_Q);
  if (rinv && q_t != 1 && v1t == 0 && path != 2 && ctx->geo.N % GS_SW == 0) gv_kmax = std::min(gv_kmax, GQ_KMIN - 1);
  if (r && k <= gv_kmax && ctx->geo.N % GV_SW == 0 && path != 3 && path != 1) {
    const double* tv = rinv ? rinv : ctx->ident + ident_offset(KP / 16);
    const int v1min = v1t > 0 ? std::max(7, v1t) : GV1_KMIN;
    const bool one_pt = k >= v1min && v1t >= 0;
    const int64_t nstrips = ctx->geo.N / (one_pt ? 64 : GV_SW);
    const int64_t nrows = ctx->geo.nrows;
    // about 8 waves per CU, whole row ranges per strip
    int64_t nranges = std::max<int64_t>(1, std::min<int64_t>(nrows, int64_t(DECOMP_CUS) * 8 / nstrips));
    const int rpr_t = tuning(ctx, GNK_TUNE_GRAM_RPR);
    // segments: the decomposition of a one-segment slab, in every segment (0: this grid cannot, per rank)
    const int64_t rpr_s = seg_on(ctx) ? seg_rpr(ctx->seg, std::max<int64_t>(1, std::min<int64_t>(
                                                    ctx->seg, int64_t(DECOMP_CUS) * 8 / nstrips)), nstrips,
                                                BLOCK / 64)
                                      : 0;
    const int64_t rpr = rpr_s > 0 ? rpr_s : rpr_t > 0 ? int64_t(rpr_t) : (nrows + nranges - 1) / nranges;
    if (seg_on(ctx) && rpr_s <= 0) ++ctx->seg_fallbacks;
    nranges = (nrows + rpr - 1) / rpr;
    const int64_t nwaves = nstrips * nranges;
    const int64_t nblk = (nwaves + BLOCK / 64 - 1) / (BLOCK / 64);
    const int NT = (k + 1) * (k + 2) / 2;
    if (nblk > (1 << 20) || size_t(nblk) * NT > SCRATCH_DOUBLES - size_t(NT))
      return fail(ctx, "gram: scratch too small (valu)");
    const int64_t nown = nrows * ctx->geo.N;
    TimedLaunch tlv(ctx, GNK_TIMER_GRAM, 8.0 * double(nown) * double(k + 2));
#define GRAMV(KV)                                                                                            \
  hipLaunchKernelGGL((k_gram_v<KV>), dim3(unsigned(nblk)), dim3(BLOCK), 0, ctx->stream, u, V, ldv, tv, KP, r, \
                     ctx->geo, ctx->coef, rpr, ctx->scratch)
#define GRAMV1(KV)                                                                                            \
  hipLaunchKernelGGL((k_gram_v1<KV>), dim3(unsigned(nblk)), dim3(BLOCK), 0, ctx->stream, u, V, ldv, tv, KP, r, \
                     ctx->geo, ctx->coef, rpr, ctx->scratch)
    if (one_pt) {
      if (k == 7) GRAMV1(7); else if (k == 8) GRAMV1(8); else GRAMV1(9);
    } else {
      switch (k) {
        case 1: GRAMV(1); break;
        case 2: GRAMV(2); break;
        case 3: GRAMV(3); break;
        case 4: GRAMV(4); break;
        case 5: GRAMV(5); break;
        case 6: GRAMV(6); break;
        case 7: GRAMV(7); break;
        case 8: GRAMV(8); break;
        default: return fail(ctx, "gram: VALU pass beyond k = 8 needs the one-point kernel");
      }
    }
#undef GRAMV1
#undef GRAMV
    tlv.done();
    int rcv = check_launch(ctx, "gram_v");
    if (rcv) return rcv;
    double* red = ctx->scratch + (SCRATCH_DOUBLES - size_t(NT));
    if (rpr_s > 0) {
      if (size_t(nblk) * NT > SEG_WS) return fail(ctx, "gram: scratch too small (valu, segments)");
      // a block is BLOCK / 64 consecutive waves = tiles (range-major): a segment's blocks are contiguous
      rcv = sreduce(ctx, ctx->scratch, int((ctx->seg / rpr) * nstrips / (BLOCK / 64)), NT, int64_t(NT), NT, 0,
                    nullptr, red);
    } else {
      rcv = wreduce(ctx, ctx->scratch, int(nblk), NT, int64_t(NT), NT, 0, nullptr, red);
    }
    if (rcv) return rcv;
    hipLaunchKernelGGL(k_gram_scatter_v, dim3(1), dim3(64), 0, ctx->stream, red, k + 1, KP, G_out);
    return check_launch(ctx, "gram scatter (valu)");
  }
  // staged kernel (measured faster than the chunked / marching kernels for the preconditioned
  // pass from k = 4 up; the marching kernel stays faster for the plain pass);
  // tuning GNK_TUNE_GRAM_PATH 1 forces it for every pass (tests), 2 disables it
  // the 4x4x4-block pass (k_gram_q) instances: column groups x DMA instructions per wave and row
  auto gq_inst = [](int ng, int L) {
    return (ng == 2 && L <= 2) || (ng == 3 && L == 2) || (ng == 4 && (L == 2 || L == 3)) || (ng == 5 && L == 3) ||
           (ng == 6 && (L == 3 || L == 4)) || (ng == 7 && L == 4) || (ng == 8 && (L == 4 || L == 5));
  };
  // preconditioned passes with k = 21..GQ_KMAX: k_gram_q too (4 ring slots, one workgroup per CU), instead of the
  // chunked k_gram_w
  const bool qwide = rinv && q_t != 1 && path != 2 && k > GS_KMAX && k <= GQ_KMAX &&
                     gq_inst((k + 3) / 4, (k + 1 + (r ? 1 : 0) + 1 + GS_NW - 1) / GS_NW);
  if (path != 2 && (path == 1 || (rinv && k >= 4)) && (k <= GS_KMAX || qwide) && ctx->geo.N % GS_SW == 0) {
    const int nbs = k <= 16 ? 1 : 2;                        // MFMA transform blocks of the V columns
    const int nrow = k + 1 + (r ? 1 : 0);
    const int L = (nrow + 1 + GS_NW - 1) / GS_NW;
    // ring depth and occupancy: one column block (k <= 16): 4 slots (the batched jdiag of EB), two blocks
    // per CU (the ring fits 80 KB; every such instance stays within the 128 VGPRs of 4 waves per SIMD);
    // two column blocks: 5 slots, one block per CU.  tuning GNK_TUNE_GRAM_RING 4 / 5 forces a depth
    // (tooling A/B; 5 slots compute one jdiag per row step).
    // Deeper rings at one block per CU (6 / 8 slots, profiles/round3/ring_sweep.jsonl) were no faster:
    // the pass is not DMA-latency bound.
    const int ring_env = tuning(ctx, GNK_TUNE_GRAM_RING);
    // ring rows (V columns, u, r) + the halo row, each R slots of gs_ss(R) doubles
    auto ring_bytes = [&](int R) { return size_t(nrow + 1) * R * gs_ss(R) * sizeof(double); };
    const size_t half_lds = 80 * 1024;
    // (4 slots: one jdiag per lane every 4 rows, EB; two column blocks run one workgroup per CU, where
    // 5 slots -- a row in flight across each barrier -- measured faster: profiles/round3/gram_eb.jsonl)
    int ring = nbs == 1 ? 4 : 5;
    if (ring_env == 4 || ring_env == 5) ring = ring_env;
    if (k > GS_KMAX) ring = 4;
    if (ring_bytes(ring) > 160 * 1024) ring = 4;
    const size_t lds = ring_bytes(ring);
    const bool two_wg = lds <= half_lds;                      // 4 waves per SIMD: VGPRs capped at 128
    if ((L <= 4 || k > GS_KMAX) && lds <= 160 * 1024) {
      const double* rv = rinv ? rinv : ctx->ident + ident_offset(KP / 16);
      // 4-column k-steps of the last transform block
      const int ksl = ((k - 16 * (nbs - 1)) + 3) / 4;
      // two blocks, 5-slot ring: the lead columns' sums on 4x4x4 MFMA for tails of >= GS_TM_MIN columns
      // (GNK_TUNE_GRAM_TM 1: never, 2: every tail)
      const int tm_t = tuning(ctx, GNK_TUNE_GRAM_TM);
      const int tm = nbs == 2 && ring == 5 && tm_t != 1 && (tm_t == 2 || k - 16 >= GS_TM_MIN) ? 1 : 0;
      const int nacc = tm ? nbs + 3 : gs_nacc(nbs, ksl);
      // the 4x4x4-block form (k_gram_q) for k >= GQ_KMIN: NG = ceil(k / 4) column groups, the ring depth chosen
      // above (4 slots up to 16 columns, 5 above); GNK_TUNE_GRAM_Q 1: never, 2: from k = 5 (k = 5..7 measured
      // 1.03-1.08 ms against the VALU kernel's 0.66-0.87)
      const int ng = (k + 3) / 4;
      const bool qinst = gq_inst(ng, L);
      const bool useq = q_t != 1 && k >= (q_t == 2 ? 5 : GQ_KMIN) && qinst &&
                        (ng == 5 || ring == 4);
      const int PL = useq ? gq_pl(ng) : 256 + 64 * nacc;
      const int wgpc = std::max(1, std::min(2, int((160 * 1024) / lds)));
      const int64_t nstrips = ctx->geo.N / GS_SW;
      const int64_t nrows = ctx->geo.nrows;
      int64_t nranges = std::max<int64_t>(1, std::min<int64_t>(nrows, int64_t(DECOMP_CUS) * wgpc / nstrips));
      const int rpr_t = tuning(ctx, GNK_TUNE_GRAM_RPR);
      const int64_t rpr_s = seg_on(ctx) ? seg_rpr(ctx->seg, std::max<int64_t>(1, std::min<int64_t>(
                                                      ctx->seg, int64_t(DECOMP_CUS) * wgpc / nstrips)), nstrips, 1)
                                        : 0;
      const int64_t rpr = rpr_s > 0 ? rpr_s : rpr_t > 0 ? int64_t(rpr_t) : (nrows + nranges - 1) / nranges;
      if (seg_on(ctx) && rpr_s <= 0) ++ctx->seg_fallbacks;
      nranges = (nrows + rpr - 1) / rpr;
      const int plog = rpr_s > 0 ? 1 : 0;             // partials at the logical (range, strip) tile
      const int64_t nwg = nstrips * nranges;
      if (nwg > (1 << 20) || size_t(nwg) * PL > SCRATCH_DOUBLES - size_t(PL))
        return fail(ctx, "gram: scratch too small (staged)");
      const int64_t nown = nrows * ctx->geo.N;
      TimedLaunch tls(ctx, GNK_TIMER_GRAM, 8.0 * double(nown) * double(k + 1 + (r ? 1 : 0)));
#define GRAMS_RW(NBV, LV, KV, TV, RV, WV)                                                                     \
  hipLaunchKernelGGL((k_gram_s<NBV, LV, KV, TV, RV, WV>), dim3(unsigned(nwg)), dim3(64 * GS_NW), lds, ctx->stream, u, \
                     V, ldv, k, rv, KP, r, ctx->geo, ctx->coef, rpr, ctx->scratch, plog)
#define GRAMS(NBV, LV, KV)                                                 \
  do {                                                                     \
    if (ring == 4 && two_wg) GRAMS_RW(NBV, LV, KV, 0, 4, 4);               \
    else if (ring == 4) GRAMS_RW(NBV, LV, KV, 0, 4, 2);                    \
    else if (two_wg) GRAMS_RW(NBV, LV, KV, 0, 5, 4);                       \
    else GRAMS_RW(NBV, LV, KV, 0, 5, 2);                                   \
  } while (0)
#define GRAMS_TR(LV, TV)                                                                                      \
  do {                                                                                                        \
    if (ring == 4) GRAMS_RW(2, LV, 1, TV, 4, 2);                                                              \
    else if (tm)                                                                                              \
      hipLaunchKernelGGL((k_gram_s<2, LV, 1, TV, 5, 2, true>), dim3(unsigned(nwg)), dim3(64 * GS_NW), lds,      \
                         ctx->stream, u, V, ldv, k, rv, KP, r, ctx->geo, ctx->coef, rpr, ctx->scratch, plog); \
    else GRAMS_RW(2, LV, 1, TV, 5, 2);                                                                        \
  } while (0)
#define GRAMS_T(LV)                                                                              \
  do {                                                                                           \
    if (k == 17) GRAMS_TR(LV, 1); else if (k == 18) GRAMS_TR(LV, 2);                             \
    else if (k == 19) GRAMS_TR(LV, 3); else GRAMS_TR(LV, 4);                                     \
  } while (0)
#define GRAMS_K(NBV, LV)                                                    \
  do {                                                                      \
    if (ksl == 1) GRAMS(NBV, LV, 1); else if (ksl == 2) GRAMS(NBV, LV, 2);  \
    else if (ksl == 3) GRAMS(NBV, LV, 3); else GRAMS(NBV, LV, 4);           \
  } while (0)
#define GRAMQ(NGV, LV, RV, WV)                                                                                 \
  hipLaunchKernelGGL((k_gram_q<NGV, LV, RV, WV>), dim3(unsigned(nwg)), dim3(64 * GS_NW), lds, ctx->stream, u, V, ldv, \
                     k, rv, KP, r, ctx->geo, ctx->coef, rpr, ctx->scratch, plog)
      if (useq) {
        if (ng == 5) { if (ring == 5) GRAMQ(5, 3, 5, 2); else GRAMQ(5, 3, 4, 2); }
        else if (ng == 6) { if (L == 3) GRAMQ(6, 3, 4, 2); else GRAMQ(6, 4, 4, 2); }
        else if (ng == 7) GRAMQ(7, 4, 4, 2);
        else if (ng == 8) { if (L == 4) GRAMQ(8, 4, 4, 2); else GRAMQ(8, 5, 4, 2); }
        else if (ng == 2 && L == 1) { if (two_wg) GRAMQ(2, 1, 4, 4); else GRAMQ(2, 1, 4, 2); }
        else if (ng == 2) { if (two_wg) GRAMQ(2, 2, 4, 4); else GRAMQ(2, 2, 4, 2); }
        else if (ng == 3) { if (two_wg) GRAMQ(3, 2, 4, 4); else GRAMQ(3, 2, 4, 2); }
        else if (L == 2) { if (two_wg) GRAMQ(4, 2, 4, 4); else GRAMQ(4, 2, 4, 2); }
        else { if (two_wg) GRAMQ(4, 3, 4, 4); else GRAMQ(4, 3, 4, 2); }
      } else if (nbs == 1) {
        if (L == 1) GRAMS_K(1, 1); else if (L == 2) GRAMS_K(1, 2); else if (L == 3) GRAMS_K(1, 3); else GRAMS_K(1, 4);
      } else {
        if (L == 3) GRAMS_T(3); else GRAMS_T(4);      // k = 17..20: one tail k-step, k - 16 tail columns
      }
#undef GRAMQ
#undef GRAMS_T
#undef GRAMS_TR
#undef GRAMS_K
#undef GRAMS
#undef GRAMS_RW
      tls.done();
      int rcs = check_launch(ctx, "gram_s");
      if (rcs) return rcs;
      double* red = ctx->scratch + (SCRATCH_DOUBLES - size_t(PL));
      if (plog) {
        if (size_t(nwg) * PL > SEG_WS) return fail(ctx, "gram: scratch too small (staged, segments)");
        rcs = sreduce(ctx, ctx->scratch, int((ctx->seg / rpr) * nstrips), PL, int64_t(PL), PL, 0, nullptr, red);
      } else {
        rcs = wreduce(ctx, ctx->scratch, int(nwg), PL, int64_t(PL), PL, 0, nullptr, red);
      }
      if (rcs) return rcs;
      if (useq)
        hipLaunchKernelGGL(k_gram_scatter_q, dim3((KP * KP + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, ctx->stream, red, ng,
                           k, r ? 1 : 0, KP, G_out);
      else
        hipLaunchKernelGGL(k_gram_scatter_s, dim3(4), dim3(BLOCK), 0, ctx->stream, red, nbs, nacc, k, r ? 1 : 0, KP,
                           tm, G_out);
      return check_launch(ctx, "gram scatter (staged)");
    }
  }
  // the wide passes below reduce over their own slab decomposition (not segmented)
  if (seg_on(ctx)) ++ctx->seg_fallbacks;
  // 3..7 column blocks on a grid of 32-point strips: k_gram_x (marching, RinvAug in VGPRs); tuning
  // GNK_TUNE_GRAM_WIDE 3 keeps the pair-split k_gram below for 5..7 blocks, 4 takes k_gram_x from 2 blocks,
  // 5 from 5 blocks (tooling A/B).  At 2 blocks (k = 21..31) the barrier-free chunked kernel stays 1.4x faster
  // (profiles/round5/gram_x_blocks_ab.jsonl); at 3 / 4 blocks k_gram_x at two workgroups per CU beats the
  // chunked / prefetching kernels (8192^2, k = 47 / 63: 12.2 / 20.3 vs 13.5 / 24.4 ms) and is flat in k.
  const int wide_t = tuning(ctx, GNK_TUNE_GRAM_WIDE);
  const int xmin = wide_t == 4 ? 2 : wide_t == 5 ? 5 : 3;
  if (nb >= xmin && nb <= 7 && ctx->geo.N % GX_T == 0 && ldv % 2 == 0 && !(wide_t == 3 && nb >= 5)) {
    const size_t ldsx = size_t(2) * GX_T * (KP + 1) * 8 + size_t(2) * GX_T * 8;    // W, Y tiles + jdiag rows
    if (size_t(4 * ((P + 3) / 4)) * 256 * 8 > ldsx) return fail(ctx, "gram: reduction staging does not fit (x)");
    const int64_t nstrips = ctx->geo.N / GX_T;
    const int64_t nrows = ctx->geo.nrows;
    // a persistent grid of the resident workgroups over (row range, strip) items; items = lcm(strips,
    // workgroups) when the rows allow, so every workgroup gets the same number
    // 8-wave workgroups, the fixed grid of GRAMX_PER_CU: one per CU at 5..7 blocks (marching rows, B fragments,
    // pair tiles: ~2 waves per SIMD), two at 2..4
    const int64_t nwg = int64_t(GRAMX_PER_CU[nb]) * DECOMP_CUS;
    const size_t ldsx_l = std::min<size_t>(160 * 1024, ldsx + decomp_lds(ctx));
    int64_t gcd = nstrips, bb = nwg;
    while (bb) { const int64_t t2 = gcd % bb; gcd = bb; bb = t2; }
    int64_t nranges = std::max<int64_t>(1, std::min<int64_t>(nrows, nwg / gcd));
    const int64_t rpr = (nrows + nranges - 1) / nranges;
    nranges = (nrows + rpr - 1) / rpr;
    const int64_t nitems = nstrips * nranges;
    const int PGx = 4 * ((P + 3) / 4);
    if (nwg > (1 << 20) || size_t(nwg) * PGx * 256 > SCRATCH_DOUBLES) return fail(ctx, "gram: scratch too small (x)");
    const int64_t nown = nrows * ctx->geo.N;
    TimedLaunch tlx(ctx, GNK_TIMER_GRAM, 8.0 * double(nown) * double(k + 1 + (r ? 1 : 0)));
#define GRAMX(NBV)                                                                                                \
  hipLaunchKernelGGL(k_gram_x<NBV>, dim3(unsigned(nwg)), dim3(64 * GX_NW), ldsx_l, ctx->stream, u, V, ldv, k, rinv, r, \
                     ctx->geo, ctx->coef, rpr, nitems, ctx->scratch)
    if (nb == 2) GRAMX(2); else if (nb == 3) GRAMX(3); else if (nb == 4) GRAMX(4);
    else if (nb == 5) GRAMX(5); else if (nb == 6) GRAMX(6); else GRAMX(7);
#undef GRAMX
    tlx.done();
    int rcx = check_launch(ctx, "gram_x");
    if (rcx) return rcx;
    (void)hipMemsetAsync(G_out, 0, size_t(KP) * KP * sizeof(double), ctx->stream);
    hipLaunchKernelGGL(k_gram_reduce, dim3((P * 256 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, ctx->stream, ctx->scratch,
                       int(nwg), P, PGx, KP, G_out);
    return check_launch(ctx, "gram reduce (x)");
  }
  if (KP <= 64) {
    // wave-independent streaming kernel
    // chunk height: 64 rows for one column block, 32 rows above (LDS tile 32 x (KP+1) per wave)
    const int chv = KP <= 32 ? 64 : 32;
    const int nwave = 4;
    size_t ldsw = size_t(nwave) * chv * (KP + 1) * 8 + (rinv ? size_t(KP) * KP * 8 : 0);
    ldsw = std::max(ldsw, size_t(P) * 256 * 8);
    ldsw = (ldsw + 15) & ~size_t(15);
    if (ldsw > 160 * 1024) return fail(ctx, "gram: LDS tile too large");
    const int64_t nown = ctx->geo.nrows * ctx->geo.N;
    const int64_t nch = (nown + chv - 1) / chv;
    const int wg_per_cu = std::max<int>(1, std::min<int>(8, int((160 * 1024) / ldsw)));
    int64_t nblk = std::min<int64_t>((nch + nwave - 1) / nwave, int64_t(DECOMP_CUS) * wg_per_cu);
    nblk = std::max<int64_t>(nblk, 1);
    if (size_t(nblk) * P * 256 > SCRATCH_DOUBLES) return fail(ctx, "gram: scratch too small");
    const int bc = chv == 64 ? (nb == 1 ? 2 : 4) : 2;
    // marching kernel: NB <= 2, strips of 64 (NB = 1) / 32 (NB = 2) columns, <= 8 columns per lane
    const int chm = nb == 1 ? 64 : 32;
    const int64_t nstrips = ctx->geo.N / chm;
    // (NB = 2 with the in-place transform keeps too few waves resident to win: chunked kernel)
    if ((nb == 1 || (nb == 2 && !rinv)) && ctx->geo.N % chm == 0 &&
        k <= 8 * (64 / (chm / 2))) {
      const int nwm = 4;
      size_t ldsm = size_t(nwm) * chm * (KP + 1) * 8 + (rinv ? size_t(KP) * KP * 8 : 0);
      ldsm = std::max(ldsm, size_t(P) * 256 * 8);
      ldsm = (ldsm + 15) & ~size_t(15);
      const int wgm = std::max<int>(1, std::min<int>(8, int((160 * 1024) / ldsm)));
      int64_t nbm = int64_t(DECOMP_CUS) * wgm;
      // whole number of row ranges per strip, at least one wave per strip
      int64_t nwv = nbm * nwm;
      if (nwv >= nstrips) {
        nwv = (nwv / nstrips) * nstrips;
        nbm = nwv / nwm;
        if (nbm * nwm == nwv && nbm >= 1) {
          TimedLaunch tlm(ctx, GNK_TIMER_GRAM, 8.0 * double(nown) * double(k + 1 + (r ? 1 : 0)));
          const int cgm = 64 / (chm / 2);
          const int mcn = (k + cgm - 1) / cgm;      // columns per lane
#define GRAMM(NBV, CHV, MCV)                                                                                   \
  hipLaunchKernelGGL((k_gram_m<NBV, CHV, MCV>), dim3(unsigned(nbm)), dim3(64 * nwm), ldsm, ctx->stream, u, V, ldv, \
                     k, rinv, r, ctx->geo, ctx->coef, ctx->scratch)
          if (nb == 1) {
            if (mcn <= 2) GRAMM(1, 64, 2);
            else if (mcn <= 4) GRAMM(1, 64, 4);
            else GRAMM(1, 64, 8);
          } else {
            if (mcn <= 4) GRAMM(2, 32, 4);
            else if (mcn <= 6) GRAMM(2, 32, 6);
            else GRAMM(2, 32, 8);
          }
#undef GRAMM
          tlm.done();
          int rcm = check_launch(ctx, "gram_m");
          if (rcm) return rcm;
          (void)hipMemsetAsync(G_out, 0, size_t(KP) * KP * sizeof(double), ctx->stream);
          double* red = ctx->scratch + (SCRATCH_DOUBLES - size_t(P) * 256);
          rcm = wreduce(ctx, ctx->scratch, int(nbm), P * 256, int64_t(P) * 256, P * 256, 0, nullptr, red);
          if (rcm) return rcm;
          hipLaunchKernelGGL(k_gram_scatter, dim3((P * 256 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, ctx->stream, red, P,
                             KP, G_out);
          return check_launch(ctx, "gram scatter");
        }
      }
    }
    // prefetching kernel for NB = 4 (k_gram_w keeps one wave per SIMD there: 98.5 KB of LDS per
    // block; at 8192^2, k = 51 / 61 with P^-1 and r: 23.0 / 24.5 ms vs 31.4 / 33.4 ms).  For NB <= 3
    // k_gram_w runs two waves per SIMD and stays ahead (k = 33: 12.4 vs 16.7 ms), so it keeps those.
    // 16-row chunks (less LDS and fewer registers per wave) and two waves per SIMD measured slower
    // for every NB (k = 51: 24.4 ms).  Tuning GNK_TUNE_GRAM_WIDE 1 / 2: never / also for NB = 2, 3
    const int wide = tuning(ctx, GNK_TUNE_GRAM_WIDE);
    if (wide != 1 && (nb == 4 || (wide == 2 && nb >= 2))) {
      constexpr int chp = 32;
      size_t ldsp = size_t(nwave) * chp * (KP + 1) * 8 + (rinv ? size_t(KP) * KP * 8 : 0);
      ldsp = std::max(ldsp, size_t(P) * 256 * 8);
      ldsp = (ldsp + 15) & ~size_t(15);
      const int64_t nchp = (nown + chp - 1) / chp;
      const int wgp = std::max<int>(1, std::min<int>(8, int((160 * 1024) / ldsp)));
      int64_t nbp = std::min<int64_t>((nchp + nwave - 1) / nwave, int64_t(DECOMP_CUS) * wgp);
      nbp = std::max<int64_t>(nbp, 1);
      if (size_t(nbp) * P * 256 > SCRATCH_DOUBLES) return fail(ctx, "gram: scratch too small");
      TimedLaunch tlp(ctx, GNK_TIMER_GRAM, 8.0 * double(nown) * double(k + 1 + (r ? 1 : 0)));
#define GRAMWP(NBV)                                                                                    \
  hipLaunchKernelGGL((k_gram_wp<NBV, chp>), dim3(unsigned(nbp)), dim3(64 * nwave), ldsp, ctx->stream, u, V, ldv, \
                     k, rinv, r, ctx->geo, ctx->coef, nchp, ctx->scratch)
      if (nb == 2) GRAMWP(2);
      else if (nb == 3) GRAMWP(3);
      else GRAMWP(4);
#undef GRAMWP
      tlp.done();
      int rcp = check_launch(ctx, "gram_wp");
      if (rcp) return rcp;
      (void)hipMemsetAsync(G_out, 0, size_t(KP) * KP * sizeof(double), ctx->stream);
      double* red = ctx->scratch + (SCRATCH_DOUBLES - size_t(P) * 256);
      rcp = wreduce(ctx, ctx->scratch, int(nbp), P * 256, int64_t(P) * 256, P * 256, 0, nullptr, red);
      if (rcp) return rcp;
      hipLaunchKernelGGL(k_gram_scatter, dim3((P * 256 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, ctx->stream, red, P, KP,
                         G_out);
      return check_launch(ctx, "gram scatter");
    }
    TimedLaunch tl(ctx, GNK_TIMER_GRAM, 8.0 * double(nown) * double(k + 1 + (r ? 1 : 0)));
#define GRAMW1(NBV, BCV, CHV) hipLaunchKernelGGL((k_gram_w<NBV, BCV, CHV>), dim3(unsigned(nblk)), dim3(64 * nwave), \
                                                 ldsw, ctx->stream, u, V, ldv, k, rinv, r, ctx->geo, ctx->coef,     \
                                                 nch, ctx->scratch)
#define GRAMW(PP)                                                  \
  do {                                                             \
    if (chv == 64) {                                               \
      if (bc == 2) GRAMW1(PP, 2, 64); else GRAMW1(PP, 4, 64);      \
    } else {                                                       \
      if (bc == 1) GRAMW1(PP, 1, 32); else GRAMW1(PP, 2, 32);      \
    }                                                              \
  } while (0)
    if (nb == 1) GRAMW(1);
    else if (nb == 2) GRAMW(2);
    else if (nb == 3) GRAMW(3);
    else GRAMW(4);
#undef GRAMW
#undef GRAMW1
    tl.done();
    int rc = check_launch(ctx, "gram_w");
    if (rc) return rc;
    (void)hipMemsetAsync(G_out, 0, size_t(KP) * KP * sizeof(double), ctx->stream);
    // partials [block][P * 256] -> red[P * 256] (scratch tail) -> symmetric G
    double* red = ctx->scratch + (SCRATCH_DOUBLES - size_t(P) * 256);
    rc = wreduce(ctx, ctx->scratch, int(nblk), P * 256, int64_t(P) * 256, P * 256, 0, nullptr, red);
    if (rc) return rc;
    hipLaunchKernelGGL(k_gram_scatter, dim3((P * 256 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, ctx->stream, red, P, KP,
                       G_out);
    return check_launch(ctx, "gram scatter");
  }
  const int rowsplit = P <= PPW_MAX ? 1 : 0;
  // pair-split: the P pair tiles spread evenly over the 4 waves (PPW = ceil(P / 4), instantiated up
  // to PPW_MAX; was 10 per wave, which left one wave of four idle at P = 28)
  int ppw = PPW_MAX;
  if (!rowsplit) {
    const int want = (P + 3) / 4;
    ppw = want <= 4 ? 4 : want <= 6 ? 6 : want <= 7 ? 7 : want <= 9 ? 9 : PPW_MAX;
  }
  const int groups = rowsplit ? 1 : (P + 4 * ppw - 1) / (4 * ppw);
  // tile rows: LDS tile <= ~40 KB for small KP (several WGs per CU), 64 rows otherwise
  int T = 256;
  while (T > 64 && size_t(T) * (KP + 1) * 8 > 40 * 1024) T >>= 1;
  int logT = 0;
  while ((1 << logT) < T) ++logT;
  const size_t tile_b = size_t(T) * (KP + 1) * 8;
  const int rinv_in_lds = rinv && tile_b + size_t(KP) * KP * 8 <= 160 * 1024 ? 1 : 0;
  size_t lds = tile_b + (rinv_in_lds ? size_t(KP) * KP * 8 : 0);
  lds = (lds + 15) & ~size_t(15);
  if (rowsplit && size_t(P) * 256 > size_t(T) * (KP + 1)) return fail(ctx, "gram: reduction staging does not fit");
  if (lds > 160 * 1024) return fail(ctx, "gram: k too large for the LDS tile");
  const int64_t nown = ctx->geo.nrows * ctx->geo.N;
  const int64_t ntiles = (nown + T - 1) / T;
  const int wg_per_cu = std::max<int>(1, std::min<int>(4, int((160 * 1024) / lds)));
  int64_t nblk = std::min<int64_t>(ntiles, int64_t(DECOMP_CUS) * wg_per_cu);
  nblk = std::max<int64_t>(nblk, 1);
  const size_t per_group_pairs = rowsplit ? P : 4 * ppw;
  if (size_t(nblk) * groups * per_group_pairs * 256 > SCRATCH_DOUBLES) return fail(ctx, "gram: scratch too small");
  // algorithmic bytes: k basis columns + u (+ r), each 8 bytes per owned point
  TimedLaunch tl(ctx, GNK_TIMER_GRAM, 8.0 * double(nown) * double(k + 1 + (r ? 1 : 0)));
#define GRAM_LAUNCH(PP)                                                                                    \
  hipLaunchKernelGGL(k_gram<PP>, dim3(unsigned(nblk), unsigned(groups)), dim3(BLOCK), lds, ctx->stream, u, V, ldv, \
                     k, rinv, r, ctx->geo, ctx->coef, T, logT, KP, P, rowsplit, ntiles, rinv_in_lds, ctx->scratch)
  if (!rowsplit) {
    if (ppw == 4) GRAM_LAUNCH(4);
    else if (ppw == 6) GRAM_LAUNCH(6);
    else if (ppw == 7) GRAM_LAUNCH(7);
    else if (ppw == 9) GRAM_LAUNCH(9);
    else GRAM_LAUNCH(PPW_MAX);
  } else if (P == 1) GRAM_LAUNCH(1);
  else if (P <= 3) GRAM_LAUNCH(3);
  else if (P <= 6) GRAM_LAUNCH(6);
  else GRAM_LAUNCH(PPW_MAX);
#undef GRAM_LAUNCH
  tl.done();
  int rc = check_launch(ctx, "gram");
  if (rc) return rc;
  (void)hipMemsetAsync(G_out, 0, size_t(KP) * KP * sizeof(double), ctx->stream);
  hipLaunchKernelGGL(k_gram_reduce, dim3((P * 256 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, ctx->stream, ctx->scratch,
                     int(nblk), P, int(per_group_pairs), KP, G_out);
  return check_launch(ctx, "gram reduce");
}

// ---------------------------------------------------------------- generic problems (flat vectors)
// No gnk_set_bratu needed: explicit lengths, a flat geometry (one "row" of n points).

#define FLAT_DISPATCH(VEC_, KERNEL, L, ...)                                                            \
  do {                                                                                                \
    if ((VEC_) == 2) hipLaunchKernelGGL(KERNEL<2>, L.grid, dim3(BLOCK), 0, ctx->stream, __VA_ARGS__);  \
    else hipLaunchKernelGGL(KERNEL<1>, L.grid, dim3(BLOCK), 0, ctx->stream, __VA_ARGS__);              \
  } while (0)

int gnk_flat_gemv(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* c, double* x, int64_t n) {
  if (!ctx_ok(ctx)) return -1;
  if (k < 1 || n < 1) return fail(ctx, "flat_gemv: k < 1 or n < 1");
  const int vec = flat_vec(n, ldv);
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec, 1 << 30);
  FLAT_DISPATCH(vec, k_gemv, L, V, ldv, k, c, x, geo, L.lr0, L.nlr);
  return check_launch(ctx, "flat_gemv");
}

int gnk_flat_gemv_t(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* g, int64_t n, double* h_out) {
  if (!ctx_ok(ctx)) return -1;
  if (k < 1 || n < 1) return fail(ctx, "flat_gemv_t: k < 1 or n < 1");
  constexpr int KCT = 8;
  const int nchunk = (k + KCT - 1) / KCT;
  const int vec = flat_vec(n, ldv);
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec, std::max(64, 4096 / nchunk));
  L.grid.z = nchunk;
  const int nblk = L.grid.x;
  if (size_t(nblk) * nchunk * KCT > SCRATCH_DOUBLES) return fail(ctx, "flat_gemv_t: scratch too small");
  if (vec == 2)
    hipLaunchKernelGGL((k_gemv_t<2, KCT>), L.grid, dim3(BLOCK), 0, ctx->stream, V, ldv, k, g, geo, L.lr0, L.nlr,
                       ctx->scratch);
  else
    hipLaunchKernelGGL((k_gemv_t<1, KCT>), L.grid, dim3(BLOCK), 0, ctx->stream, V, ldv, k, g, geo, L.lr0, L.nlr,
                       ctx->scratch);
  int rc = check_launch(ctx, "flat_gemv_t");
  if (rc) return rc;
  return wreduce(ctx, ctx->scratch, nblk, k, KCT, KCT, int64_t(nblk) * KCT, nullptr, h_out);
}

int gnk_flat_cgs_update(gnk_ctx* ctx, const double* V, int64_t ldv, int k, const double* h, double* g, int64_t n,
                        double* stats_out) {
  if (!ctx_ok(ctx)) return -1;
  if (k < 1 || n < 1) return fail(ctx, "flat_cgs_update: k < 1 or n < 1");
  const int vec = flat_vec(n, ldv);
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec);
  FLAT_DISPATCH(vec, k_cgs, L, V, ldv, k, h, g, geo, L.lr0, L.nlr, ctx->scratch);
  int rc = check_launch(ctx, "flat_cgs_update");
  if (rc) return rc;
  return reduce(ctx, ctx->scratch, int(L.grid.x), 2, 2, sum_max_flags(), stats_out);
}

int gnk_flat_stats(gnk_ctx* ctx, const double* x, int64_t n, double* stats_out) {
  if (!ctx_ok(ctx)) return -1;
  if (n < 1) return fail(ctx, "flat_stats: n < 1");
  const int vec = al16(x) ? flat_vec(n) : 1;
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec);
  FLAT_DISPATCH(vec, k_stats, L, x, geo, L.lr0, L.nlr, ctx->scratch);
  int rc = check_launch(ctx, "flat_stats");
  if (rc) return rc;
  return reduce_stats(ctx, ctx->scratch, int(L.grid.x), stats_out);
}

int gnk_flat_dot(gnk_ctx* ctx, const double* a, const double* b, int64_t n, double* out) {
  if (!ctx_ok(ctx)) return -1;
  if (n < 1) return fail(ctx, "flat_dot: n < 1");
  const int vec = flat_vec(n);
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec);
  FLAT_DISPATCH(vec, k_dot, L, a, b, geo, L.lr0, L.nlr, ctx->scratch);
  int rc = check_launch(ctx, "flat_dot");
  if (rc) return rc;
  return wreduce2(ctx, ctx->scratch, int(L.grid.x), 1, 2, out);
}

int gnk_flat_div(gnk_ctx* ctx, const double* src, double denom, double* dst, int64_t n) {
  if (!ctx_ok(ctx)) return -1;
  const int vec = (al16(src) && al16(dst)) ? flat_vec(n) : 1;
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec, 1 << 30);
  FLAT_DISPATCH(vec, k_div, L, src, denom, dst, geo, L.lr0, L.nlr);
  return check_launch(ctx, "flat_div");
}

int gnk_flat_axpy(gnk_ctx* ctx, const double* x, double alpha, const double* d, double* out, int64_t n) {
  if (!ctx_ok(ctx)) return -1;
  const int vec = (al16(x) && al16(d) && al16(out)) ? flat_vec(n) : 1;
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec, 1 << 30);
  FLAT_DISPATCH(vec, k_axpy, L, x, alpha, d, out, geo, L.lr0, L.nlr);
  return check_launch(ctx, "flat_axpy");
}

int gnk_flat_cg_update_xr(gnk_ctx* ctx, double alpha, const double* p, const double* q, double* x, double* r,
                          const double* dinv, double* z, int64_t n, double* out) {
  if (!ctx_ok(ctx)) return -1;
  const int vec = (al16(p) && al16(q) && al16(x) && al16(r) && al16(dinv) && al16(z)) ? flat_vec(n) : 1;
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec);
  FLAT_DISPATCH(vec, k_cg_xr, L, alpha, p, q, x, r, dinv, z, geo, L.lr0, L.nlr, ctx->scratch, nullptr);
  int rc = check_launch(ctx, "flat_cg_update_xr");
  if (rc) return rc;
  return wreduce2(ctx, ctx->scratch, int(L.grid.x), 2, 4, out);
}

int gnk_flat_cg_update_p(gnk_ctx* ctx, double beta, int first, const double* z, double* p, int64_t n) {
  if (!ctx_ok(ctx)) return -1;
  const int vec = (al16(z) && al16(p)) ? flat_vec(n) : 1;
  const Geo geo{n, 0, 1};
  RowLaunch L = flat_rows(n, vec, 1 << 30);
  FLAT_DISPATCH(vec, k_cg_p, L, beta, first, z, p, geo, L.lr0, L.nlr);
  return check_launch(ctx, "flat_cg_update_p");
}

int gnk_csr_spmv(gnk_ctx* ctx, int64_t nrows, const int* indptr, const int* indices, const double* data,
                 const double* x, double* y, int mode) {
  if (!ctx_ok(ctx)) return -1;
  if (nrows < 1 || !indptr || !x || !y) return fail(ctx, "csr_spmv: bad arguments");
  const int64_t nb = std::min<int64_t>((nrows + BLOCK - 1) / BLOCK, 1 << 20);
  if (mode < 0 || mode > 2) return fail(ctx, "csr_spmv: mode must be 0, 1 or 2");
  hipLaunchKernelGGL(k_csr_spmv, dim3(unsigned(nb)), dim3(BLOCK), 0, ctx->stream, nrows, indptr, indices, data, x, y,
                     mode);
  return check_launch(ctx, "csr_spmv");
}

int gnk_flat_gram(gnk_ctx* ctx, const double* W, int64_t ldw, int k, const double* rinv, int64_t ldr,
                  const double* r, int64_t m, double* G_out) {
  if (!ctx_ok(ctx)) return -1;
  if (k < 1 || m < 1) return fail(ctx, "flat_gram: k < 1 or m < 1");
  const int KP = gnk_gram_padded_dim(k, r != nullptr);
  const int nb = KP / 16;
  if (rinv && ldr != KP) return fail(ctx, "flat_gram: rinv must be the kp x kp augmented inverse (ldr == kp)");
  if (nb > 4) {
    // wide basis: Y = W RinvAug materialised in the scratch arena, then the pairwise Gram
    if (size_t(KP) * size_t(m) > SCRATCH_DOUBLES || KP > 1024) return fail(ctx, "flat_gram: basis too wide for the scratch arena");
    double* Y = ctx->scratch;
    const unsigned gx = unsigned(std::min<int64_t>((m + BLOCK - 1) / BLOCK, 1024));
    hipLaunchKernelGGL(k_flat_ytrans, dim3(gx, KP), dim3(BLOCK), 0, ctx->stream, W, ldw, k, rinv, KP, r, m, KP, Y);
    int rc = check_launch(ctx, "flat_gram ytrans");
    if (rc) return rc;
    hipLaunchKernelGGL(k_flat_syrk, dim3(KP * (KP + 1) / 2), dim3(BLOCK), 0, ctx->stream, Y, m, KP, G_out);
    return check_launch(ctx, "flat_gram syrk");
  }
  const double* rv = rinv ? rinv : ctx->ident + ident_offset(nb);
  const int P = nb * (nb + 1) / 2;
  const int64_t nchunk = (m + 15) / 16;
  const int nblk = int(std::max<int64_t>(1, std::min<int64_t>((nchunk + 3) / 4, 1024)));
  if (size_t(nblk) * P * 256 > SCRATCH_DOUBLES - size_t(P) * 256) return fail(ctx, "flat_gram: scratch too small");
  switch (nb) {
    case 1: hipLaunchKernelGGL(k_flat_gram<1>, dim3(nblk), dim3(BLOCK), 0, ctx->stream, W, ldw, k, rv, KP, r, m, ctx->scratch); break;
    case 2: hipLaunchKernelGGL(k_flat_gram<2>, dim3(nblk), dim3(BLOCK), 0, ctx->stream, W, ldw, k, rv, KP, r, m, ctx->scratch); break;
    case 3: hipLaunchKernelGGL(k_flat_gram<3>, dim3(nblk), dim3(BLOCK), 0, ctx->stream, W, ldw, k, rv, KP, r, m, ctx->scratch); break;
    default: hipLaunchKernelGGL(k_flat_gram<4>, dim3(nblk), dim3(BLOCK), 0, ctx->stream, W, ldw, k, rv, KP, r, m, ctx->scratch); break;
  }
  int rc = check_launch(ctx, "flat_gram");
  if (rc) return rc;
  (void)hipMemsetAsync(G_out, 0, size_t(KP) * KP * sizeof(double), ctx->stream);
  double* red = ctx->scratch + (SCRATCH_DOUBLES - size_t(P) * 256);
  rc = wreduce(ctx, ctx->scratch, nblk, P * 256, int64_t(P) * 256, P * 256, 0, nullptr, red);
  if (rc) return rc;
  hipLaunchKernelGGL(k_gram_scatter, dim3((P * 256 + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, ctx->stream, red, P, KP,
                     G_out);
  return check_launch(ctx, "flat_gram scatter");
}

// Row ranges of the row-marching normal matvec: the fixed grid of CGM_PER_CU (one round of its resident
// workgroups on MI355X; nbc strips of 4 waves per range), not a fixed 8 per CU -- at 5 resident workgroups per CU
// a fixed 8 is 1.6 rounds.  The p.q partials are compensated pairs (Dot2, about twice working precision, not
// exact): their bits follow this decomposition, which depends on N and the slab's rows only.
int64_t cgm_ranges(int64_t nbc, int64_t nrows) {
  return std::max<int64_t>(1, std::min<int64_t>(nrows, int64_t(CGM_PER_CU) * DECOMP_CUS / nbc));
}

int gnk_cg_normal_matvec(gnk_ctx* ctx, const double* d, const double* p, double* q, double* pq_out) {
  if (!ready(ctx)) return -1;
  int nblk;
  if (ctx->geo.N % 2 == 0 && tuning(ctx, GNK_TUNE_CG_MATVEC) != 1) {
    const int64_t nbc = (ctx->geo.N + 4 * CGM_SW - 1) / (4 * CGM_SW);
    const int64_t nrows = ctx->geo.nrows;
    int64_t nranges = cgm_ranges(nbc, nrows);
    const int64_t rpr = (nrows + nranges - 1) / nranges;
    nranges = (nrows + rpr - 1) / rpr;
    if (nbc * nranges > MAX_RED_BLOCKS) return fail(ctx, "cg_normal_matvec: grid too large");
    nblk = int(nbc * nranges);
    TimedLaunch tl(ctx, GNK_TIMER_CG_MATVEC, 24.0 * double(nrows) * double(ctx->geo.N));
    hipLaunchKernelGGL(k_cg_matvec_m<false>, dim3(unsigned(nblk)), dim3(BLOCK), decomp_lds(ctx), ctx->stream, d, p, q, ctx->geo,
                       ctx->coef, rpr, ctx->scratch, nullptr, nullptr, 0.0, 0, nullptr, 0.0, nullptr);
    tl.done();
  } else {
    RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx));
    nblk = L.grid.x * L.grid.y;
    DISPATCH_VEC(ctx, k_cg_matvec, L, 0, d, p, q, ctx->geo, ctx->coef, L.lr0, L.nlr, ctx->scratch);
  }
  int rc = check_launch(ctx, "cg_normal_matvec");
  if (rc) return rc;
  TimedLaunch ta(ctx, GNK_TIMER_CG_AUX, 0.0);
  rc = wreduce2(ctx, ctx->scratch, nblk, 1, 2, pq_out);
  ta.done();
  return rc;
}

static int cg_step_matvec(gnk_ctx* ctx, const double* d, const double* z, const double* p_in, double* p_out,
                          double* q, double beta, int first, double* x, double xalpha, const double* cst,
                          double* pq_out) {
  if (!ready(ctx)) return -1;
  if (ctx->geo.N % 2) return fail(ctx, "cg_step_matvec: N must be even (use cg_update_p + cg_normal_matvec)");
  if (!d || !z || !p_in || !p_out || !q || p_in == p_out) return fail(ctx, "cg_step_matvec: bad buffers");
  const int64_t nbc = (ctx->geo.N + 4 * CGM_SW - 1) / (4 * CGM_SW);
  const int64_t nrows = ctx->geo.nrows;
  int64_t nranges = cgm_ranges(nbc, nrows);
  const int64_t rpr = (nrows + nranges - 1) / nranges;
  nranges = (nrows + rpr - 1) / rpr;
  if (nbc * nranges > MAX_RED_BLOCKS) return fail(ctx, "cg_step_matvec: grid too large");
  const int nblk = int(nbc * nranges);
  TimedLaunch tl(ctx, GNK_TIMER_CG_MATVEC, (x ? 56.0 : 40.0) * double(nrows) * double(ctx->geo.N));
  hipLaunchKernelGGL(k_cg_matvec_m<true>, dim3(unsigned(nblk)), dim3(BLOCK), decomp_lds(ctx), ctx->stream, d, p_in, q, ctx->geo,
                     ctx->coef, rpr, ctx->scratch, z, p_out, beta, first, x, xalpha, cst);
  tl.done();
  int rc = check_launch(ctx, "cg_step_matvec");
  if (rc) return rc;
  TimedLaunch ta(ctx, GNK_TIMER_CG_AUX, 0.0);
  rc = wreduce2(ctx, ctx->scratch, nblk, 1, 2, pq_out);
  ta.done();
  return rc;
}

int gnk_cg_step_matvec(gnk_ctx* ctx, const double* d, const double* z, const double* p_in, double* p_out, double* q,
                       double beta, int first, double* x, double xalpha, double* pq_out) {
  return cg_step_matvec(ctx, d, z, p_in, p_out, q, beta, first, x, xalpha, nullptr, pq_out);
}

int gnk_cg_step_matvec_dev(gnk_ctx* ctx, const double* d, const double* z, const double* p_in, double* p_out,
                           double* q, int first, double* x, const double* state, double* pq_out) {
  if (!state) return fail(ctx, "cg_step_matvec_dev: NULL state");
  return cg_step_matvec(ctx, d, z, p_in, p_out, q, 0.0, first, x, 0.0, state, pq_out);
}

static int cg_update_xr(gnk_ctx* ctx, double alpha, const double* cst, const double* p, const double* q, double* x,
                        double* r, const double* dinv, double* z, double* out) {
  if (!ready(ctx)) return -1;
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx));
  const int nblk = L.grid.x * L.grid.y;
  // r -= alpha q, z = M r (+ x += alpha p): q, r, dinv in, r, z out (+ x, p in, x out)
  TimedLaunch tl(ctx, GNK_TIMER_CG_XR, ((x && p) ? 64.0 : 40.0) * double(ctx->geo.nrows) * double(ctx->geo.N));
  DISPATCH_VEC(ctx, k_cg_xr, L, 0, alpha, p, q, x, r, dinv, z, ctx->geo, L.lr0, L.nlr, ctx->scratch, cst);
  tl.done();
  int rc = check_launch(ctx, "cg_update_xr");
  if (rc) return rc;
  TimedLaunch ta(ctx, GNK_TIMER_CG_AUX, 0.0);
  rc = wreduce2(ctx, ctx->scratch, nblk, 2, 4, out);
  ta.done();
  return rc;
}

int gnk_cg_update_xr(gnk_ctx* ctx, double alpha, const double* p, const double* q, double* x, double* r,
                     const double* dinv, double* z, double* out) {
  return cg_update_xr(ctx, alpha, nullptr, p, q, x, r, dinv, z, out);
}

int gnk_cg_update_xr_dev(gnk_ctx* ctx, const double* state, const double* p, const double* q, double* x, double* r,
                         const double* dinv, double* z, double* out) {
  if (!state) return fail(ctx, "cg_update_xr_dev: NULL state");
  return cg_update_xr(ctx, 0.0, state, p, q, x, r, dinv, z, out);
}

int gnk_cg_scalars(gnk_ctx* ctx, const double* parts, int world, int stage, double* state) {
  if (!ready(ctx)) return -1;
  if (!parts || !state || world < 1 || stage < 0 || stage > 2) return fail(ctx, "cg_scalars: bad arguments");
  TimedLaunch ta(ctx, GNK_TIMER_CG_AUX, 0.0);
  hipLaunchKernelGGL(k_cg_scalars, dim3(1), dim3(64), 0, ctx->stream, parts, world, stage, state);
  ta.done();
  return check_launch(ctx, "cg_scalars");
}

int gnk_cg_sr_update(gnk_ctx* ctx, double alpha, double beta, int first, const double* w, double* p, double* s,
                     double* x, double* r, const double* dinv, double* u, double* out) {
  if (!ready(ctx)) return -1;
  if (!w || !p || !s || !x || !r || !u || !out) return fail(ctx, "cg_sr_update: NULL argument");
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx));
  const int nblk = L.grid.x * L.grid.y;
  DISPATCH_VEC(ctx, k_cg_sr, L, 0, alpha, beta, first, w, p, s, x, r, dinv, u, ctx->geo, L.lr0, L.nlr, ctx->scratch);
  int rc = check_launch(ctx, "cg_sr_update");
  if (rc) return rc;
  return reduce(ctx, ctx->scratch, nblk, 2, 2, nullptr, out);
}

int gnk_cg_update_p(gnk_ctx* ctx, double beta, int first, const double* z, double* p) {
  if (!ready(ctx)) return -1;
  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);
  DISPATCH_VEC(ctx, k_cg_p, L, 0, beta, first, z, p, ctx->geo, L.lr0, L.nlr);
  return check_launch(ctx, "cg_update_p");
}

int gnk_decomp_check(gnk_ctx* ctx, int* table_out, int* live_out, int capacity) {
  if (!ctx) return -1;
  std::vector<std::pair<int, const void*>> inst;      // (table workgroups per CU, kernel) in a fixed order
  std::vector<std::pair<int, size_t>> geom;           // (threads per workgroup, dynamic LDS)
  for (int v = 1; v <= 2; ++v)
    for (int p = 0; p <= 1; ++p)
      for (int kct = 1; kct <= 24; ++kct) {
        const void* fn = v == 2 ? (p ? vjpg_pick<2, true>(kct) : vjpg_pick<2, false>(kct))
                                : (p ? vjpg_pick<1, true>(kct) : vjpg_pick<1, false>(kct));
        inst.push_back({VJPG_PER_CU[v - 1][p][kct - 1], fn});
        geom.push_back({BLOCK, 0});
      }
  inst.push_back({GEMVP_PER_CU, (const void*)&k_gemv_p<1>});
  geom.push_back({BLOCK, 0});
  inst.push_back({GEMVP_PER_CU, (const void*)&k_gemv_p<2>});
  geom.push_back({BLOCK, 0});
  const void* gx[8] = {nullptr, nullptr, (const void*)&k_gram_x<2>, (const void*)&k_gram_x<3>, (const void*)&k_gram_x<4>,
                       (const void*)&k_gram_x<5>, (const void*)&k_gram_x<6>, (const void*)&k_gram_x<7>};
  for (int nb = 2; nb <= 7; ++nb) {
    const int KP = 16 * nb;
    inst.push_back({GRAMX_PER_CU[nb], gx[nb]});
    geom.push_back({64 * GX_NW, size_t(2) * GX_T * (KP + 1) * 8 + size_t(2) * GX_T * 8});
  }
  inst.push_back({CGM_PER_CU, (const void*)&k_cg_matvec_m<false>});
  geom.push_back({BLOCK, 0});
  inst.push_back({CGM_PER_CU, (const void*)&k_cg_matvec_m<true>});
  geom.push_back({BLOCK, 0});
  const int n = int(inst.size());
  for (int i = 0; i < std::min(n, capacity); ++i) {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, inst[i].second, geom[i].first, geom[i].second) != hipSuccess)
      per = -1;
    if (table_out) table_out[i] = inst[i].first;
    if (live_out) live_out[i] = per;
  }
  return n;
}

int gnk_timer_start(gnk_ctx* ctx, int kernel_id, int capacity) {
  if (!ctx) return -1;
  if (capacity < 0) return fail(ctx, "timer_start: capacity < 0");
  if (kernel_id < 1 || kernel_id > 30) return fail(ctx, "timer_start: kernel_id out of range");
  while (int(ctx->timer_ev.size()) < 2 * capacity) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return fail(ctx, "timer_start: hipEventCreate failed", -2);
    ctx->timer_ev.push_back(e);
  }
  ctx->timer_bytes.assign(capacity, 0.0);
  ctx->timer_ids.assign(capacity, 0);
  ctx->timer_mask = 1u << kernel_id;
  ctx->timer_count = 0;
  return 0;
}

int gnk_timer_add(gnk_ctx* ctx, int kernel_id) {
  if (!ctx) return -1;
  if (kernel_id < 1 || kernel_id > 30) return fail(ctx, "timer_add: kernel_id out of range");
  if (!ctx->timer_mask) return fail(ctx, "timer_add: no timer started");
  ctx->timer_mask |= 1u << kernel_id;
  return 0;
}

int gnk_timer_collect_ids(gnk_ctx* ctx, double* ms_out, double* bytes_out, int* ids_out, int capacity) {
  if (!ctx) return -1;
  const int n = std::min(capacity, ctx->timer_count);
  for (int i = 0; i < n; ++i) {
    if (hipEventSynchronize(ctx->timer_ev[2 * i + 1]) != hipSuccess) return fail(ctx, "timer_collect: sync", -2);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->timer_ev[2 * i], ctx->timer_ev[2 * i + 1]) != hipSuccess)
      return fail(ctx, "timer_collect: elapsed", -2);
    ms_out[i] = ms;
    bytes_out[i] = ctx->timer_bytes[i];
    if (ids_out) ids_out[i] = ctx->timer_ids[i];
  }
  ctx->timer_mask = 0;
  ctx->timer_count = 0;
  return n;
}

int gnk_timer_collect(gnk_ctx* ctx, double* ms_out, double* bytes_out, int capacity) {
  return gnk_timer_collect_ids(ctx, ms_out, bytes_out, nullptr, capacity);
}

int gnk_rank_sum(gnk_ctx* ctx, const double* parts, int world, int64_t n, double* out) {
  if (!ctx) return -1;
  if (world < 1 || n < 0) return fail(ctx, "rank_sum: world < 1 or n < 0");
  if (n == 0) return 0;
  if (!parts || !out) return fail(ctx, "rank_sum: NULL argument");
  const int64_t nb = std::min<int64_t>((n + BLOCK - 1) / BLOCK, 1024);
  hipLaunchKernelGGL(k_rank_sum, dim3(unsigned(nb)), dim3(BLOCK), 0, ctx->stream, parts, world, n, out);
  return check_launch(ctx, "rank_sum");
}

int gnk_lls_max_k(void) { return LS_KMAX; }

int gnk_lls_next(gnk_ctx* ctx, int k, int pending, const double* out, const double* e_try, const double* pack,
                 const double* sc, int kp_next, double* T_next, double* P_next, double* sdd_next, double* e_next,
                 double* hh_next, double* sc_next) {
  if (!ctx) return -1;
  if (k < 1 || k + 1 > LS_KMAX) return fail(ctx, "lls_next: k + 1 must be in [2, gnk_lls_max_k()]");
  if (kp_next < k + 2) return fail(ctx, "lls_next: kp_next < k + 2");
  if (!out || !e_try || !pack || !sc || !T_next || !P_next || !sdd_next || !e_next || !hh_next || !sc_next)
    return fail(ctx, "lls_next: NULL argument");
  hipLaunchKernelGGL(k_lls_next, dim3(1), dim3(256),   // 4 waves: the T / P fills are latency bound
                     0, ctx->stream, k, pending, out, e_try, pack, sc, kp_next,
                     T_next, P_next, sdd_next, e_next, hh_next, sc_next);
  return check_launch(ctx, "lls_next");
}

int gnk_lls_solve(gnk_ctx* ctx, const double* Gm, int kp, int k, const double* P, int rescale, const double* sdd,
                  const double* e, double* out, double* e_try) {
  if (!ctx) return -1;
  if (k < 1 || k > LS_KMAX) return fail(ctx, "lls_solve: k must be in [1, gnk_lls_max_k()]");
  if (kp < k + 1) return fail(ctx, "lls_solve: kp < k + 1 (G must hold the r column)");
  if (!Gm || !P || !sdd || !e || !out || !e_try) return fail(ctx, "lls_solve: NULL argument");
  // one entry per thread (k_lls_2d) by default; tuning GNK_TUNE_LLS 1 keeps the one-wave k_lls (tooling A/B,
  // the same bits)
  if (tuning(ctx, GNK_TUNE_LLS) != 1)
    hipLaunchKernelGGL(k_lls_2d, dim3(1), dim3(1024), 0, ctx->stream, Gm, kp, k, P, rescale, sdd, e, out, e_try);
  else
    hipLaunchKernelGGL(k_lls, dim3(1), dim3(64), 0, ctx->stream, Gm, kp, k, P, rescale, sdd, e, out, e_try);
  return check_launch(ctx, "lls_solve");
}

// tooling: fp64 MFMA issue-rate probe (not part of the solver)
int gnk_probe_stream(gnk_ctx* ctx, double* a, const double* b, const double* c, double s, int64_t n, int mode) {
  if (!ctx) return -1;
  if (mode < 0 || mode > 2 || n < 2 || n % 2 != 0) return fail(ctx, "probe_stream: mode in 0..2, n even >= 2");
  if (!b || (mode != 1 && !a) || (mode == 0 && !c)) return fail(ctx, "probe_stream: NULL argument");
  const int64_t n2 = n / 2;
  const int64_t blocks = (n2 + BLOCK * 4 - 1) / (BLOCK * 4);
  if (blocks > (1 << 30) || (mode == 1 && blocks * (BLOCK / 64) > int64_t(SCRATCH_DOUBLES)))
    return fail(ctx, "probe_stream: n too large");
  const double bytes = 8.0 * double(n) * (mode == 0 ? 3.0 : mode == 1 ? 1.0 : 2.0);
  TimedLaunch tl(ctx, GNK_TIMER_PROBE, bytes);
  hipLaunchKernelGGL(k_probe_stream, dim3(unsigned(blocks)), dim3(BLOCK), 0, ctx->stream, a, b, c, s, n2, mode,
                     ctx->scratch);
  tl.done();
  return check_launch(ctx, "probe_stream");
}

int gnk_probe_mfma_f64(gnk_ctx* ctx, double* out, int blocks, int iters) {
  if (!ctx) return -1;
  hipLaunchKernelGGL(k_probe_mfma, dim3(blocks), dim3(BLOCK), 0, ctx->stream, out, iters);
  return check_launch(ctx, "probe_mfma");
}

}  // extern "C"
