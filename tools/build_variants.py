"""Ablation / experiment builds of libgnk.so (tooling only: the product source is never edited).

python tools/build_variants.py NAME [NAME ...]      -> tools/_var/libgnk_NAME.so
Each variant is the product source with the text substitutions listed in VARIANTS applied (every
substitution must match, else the build stops).  Load one with GNK_LIB=tools/_var/libgnk_NAME.so.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gauss_newton_via_generalized_krylov_subspaces_amd", "csrc", "gnk_kernels.hip")
OUT = os.path.join(ROOT, "tools", "_var")   # gitignored, travels to the GPU box

_STEP_BARRIER = ("__builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(L * INF));     // row x+3 landed\n"
                 "        __builtin_amdgcn_s_barrier();")
VARIANTS = {
    # k_gram_s: no barrier at the end of a row step (wrong results; what the per-step barrier costs)
    "nobar": [(_STEP_BARRIER, "__builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(L * INF));     // row x+3 landed")],
    # k_gram_s: no exp (dn from u directly)
    "noexp": [("dn = -jdiag(cf, Lx2[ou]);                   // row x+2", "dn = -Lx2[ou];")],
    # k_gram_s: Gram step replaced by one add (transform + stencil + DMA only)
    "nogram": [("        gram(H, Lx);                                  // row x (its r is in slot x)",
                "        acc[0] += H[0][0];")],
    # k_gram_x: the transform's block chains split into two accumulators (even / odd k-steps)
    "gx2acc": [("""          d4 qa = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ab = 0; ab <= CA; ++ab)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) qa = mfma64(arow[ab * 16 + ks * 4], rA[ab][ks], qa);
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) Yt""", """          d4 qa = d4{0.0, 0.0, 0.0, 0.0}, qz = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ab = 0; ab <= CA; ++ab)
#pragma unroll
            for (int ks = 0; ks < 4; ks += 2) {
              qa = mfma64(arow[ab * 16 + ks * 4], rA[ab][ks], qa);
              qz = mfma64(arow[ab * 16 + ks * 4 + 4], rA[ab][ks + 1], qz);
            }
          qa = qa + qz;
#pragma unroll
          for (int ii = 0; ii < 4; ++ii) Yt""")],
    # k_gram_s: no VALU tail / r sums (MFMA tile only)
    "notail": [("    if (NB == 2) {\n#pragma unroll\n      for (int t = 0; t < TAIL; ++t) {",
                "    if (false) {\n#pragma unroll\n      for (int t = 0; t < TAIL; ++t) {")],
    # k_gram_v1: the next row's V / u / r loads issued one row ahead (software-pipelined march)
    "v1pf": [("    for (int64_t x = x0; x < x1; ++x, i += N) {\n      double vs[K], eo[K];\n#pragma unroll\n      for (int j = 0; j < K; ++j) {\n        const double* cp = V + j * ldv + i;\n        vs[j] = cp[N];\n        eo[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;     // only the strip's edge lanes load\n      }\n      const double dn = -jdiag(c, u[i]);\n      const double rv = r[i];\n      double a[K];", "    double vs[K], eo[K];\n#pragma unroll\n    for (int j = 0; j < K; ++j) {\n      const double* cp = V + j * ldv + i;\n      vs[j] = cp[N];\n      eo[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;\n    }\n    double uc = u[i], rv = r[i];\n    for (int64_t x = x0; x < x1; ++x, i += N) {\n      // the next row's loads are issued before this row's arithmetic (row G + x + 2 <= the last ghost row)\n      double vs2[K], eo2[K];\n#pragma unroll\n      for (int j = 0; j < K; ++j) {\n        const double* cp = V + j * ldv + i + N;\n        vs2[j] = cp[N];\n        eo2[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;\n      }\n      const double u2 = u[i + N], r2 = r[i + N];\n      const double dn = -jdiag(c, uc);\n      double a[K];"), ('        a[j] = sv;\n        vn[j] = vc[j];\n        vc[j] = vs[j];\n      }\n      gram_v_point<K>(a, rv, T, ldt, acc);\n    }', '        a[j] = sv;\n        vn[j] = vc[j];\n        vc[j] = vs[j];\n      }\n      gram_v_point<K>(a, rv, T, ldt, acc);\n#pragma unroll\n      for (int j = 0; j < K; ++j) {\n        vs[j] = vs2[j];\n        eo[j] = eo2[j];\n      }\n      uc = u2;\n      rv = r2;\n    }')],
    # k_gram_v1: the transform T staged in LDS (broadcast reads) instead of SGPRs (18 / 52 SGPR spills at K = 8 / 9)
    "v1lds": [("__global__ __launch_bounds__(BLOCK) void k_gram_v1(",
               "__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(2))) void k_gram_v1("), ("  const int eoff = edge_w ? -1 : 1;                 // the edge lanes' outer neighbour (others: unused)\n  double acc[NT];", "  const int eoff = edge_w ? -1 : 1;                 // the edge lanes' outer neighbour (others: unused)\n  __shared__ double Ts[K * K];\n  for (int t = threadIdx.x; t < K * K; t += BLOCK) Ts[t] = T[(t / K) * ldt + t % K];\n  __syncthreads();\n  double acc[NT];"), ('      gram_v_point<K>(a, rv, T, ldt, acc);\n    }\n  }\n#pragma unroll\n  for (int q = 0; q < NT; ++q) {\n    const double sq = wave_sum(acc[q]);\n    if (lane == 0) red[wave][q] = sq;\n  }\n  __syncthreads();\n  for (int q = threadIdx.x; q < NT; q += BLOCK) {\n    double sq = red[0][q];\n    for (int w = 1; w < BLOCK / 64; ++w) sq += red[w][q];\n    partial[size_t(blockIdx.x) * NT + q] = sq;\n  }\n}\n\n// packed upper triangle', '      int z = 0;\n      asm volatile("" : "+s"(z));                   // opaque 0: the LDS reads stay in the row loop\n      gram_v_point<K>(a, rv, Ts + z, K, acc);\n    }\n  }\n#pragma unroll\n  for (int q = 0; q < NT; ++q) {\n    const double sq = wave_sum(acc[q]);\n    if (lane == 0) red[wave][q] = sq;\n  }\n  __syncthreads();\n  for (int q = threadIdx.x; q < NT; q += BLOCK) {\n    double sq = red[0][q];\n    for (int w = 1; w < BLOCK / 64; ++w) sq += red[w][q];\n    partial[size_t(blockIdx.x) * NT + q] = sq;\n  }\n}\n\n// packed upper triangle')],
    # k_jvp: non-temporal stores of J v / a grid of the resident workgroups (row-strided) / both
    "jvpnt": [('      o.y = jvp_pt(c, d1, vn.y, vc.x, true, vc.y, ve, he, vs.y);\n    }\n    *reinterpret_cast<d2*>(out + li) = o;', '      o.y = jvp_pt(c, d1, vn.y, vc.x, true, vc.y, ve, he, vs.y);\n    }\n    __builtin_nontemporal_store(o, reinterpret_cast<d2*>(out + li));')],
    "jvpres": [('  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);\n  TimedLaunch tl(ctx, GNK_TIMER_JVP, 24.0 * double(ctx->geo.nrows) * double(ctx->geo.N));\n  DISPATCH_VEC(ctx, k_jvp, L, 0, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr, 0);', '  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), resident_blocks(ctx, (const void*)&k_jvp<2>));\n  TimedLaunch tl(ctx, GNK_TIMER_JVP, 24.0 * double(ctx->geo.nrows) * double(ctx->geo.N));\n  DISPATCH_VEC(ctx, k_jvp, L, 0, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr, 0);')],
    "jvpntres": [('      o.y = jvp_pt(c, d1, vn.y, vc.x, true, vc.y, ve, he, vs.y);\n    }\n    *reinterpret_cast<d2*>(out + li) = o;', '      o.y = jvp_pt(c, d1, vn.y, vc.x, true, vc.y, ve, he, vs.y);\n    }\n    __builtin_nontemporal_store(o, reinterpret_cast<d2*>(out + li));'), ('  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);\n  TimedLaunch tl(ctx, GNK_TIMER_JVP, 24.0 * double(ctx->geo.nrows) * double(ctx->geo.N));\n  DISPATCH_VEC(ctx, k_jvp, L, 0, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr, 0);', '  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), resident_blocks(ctx, (const void*)&k_jvp<2>));\n  TimedLaunch tl(ctx, GNK_TIMER_JVP, 24.0 * double(ctx->geo.nrows) * double(ctx->geo.N));\n  DISPATCH_VEC(ctx, k_jvp, L, 0, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr, 0);')],
    # k_jvp2: two grid rows per lane pass (4 v row loads per 2 output rows instead of 6)
    "jvp2r": [('template <int VEC>\n__global__ __launch_bounds__(BLOCK) void k_forward(', '// J(u) v for two grid rows per lane pass (rows lr, lr + 1; N % 128 == 0): the centre and south v rows\n// serve both outputs, so 4 v row loads per 2 output rows instead of 6; same per-point arithmetic as k_jvp\n__global__ __launch_bounds__(BLOCK) void k_jvp2(const double* __restrict__ u, const double* __restrict__ v,\n                                                double* __restrict__ out, Geo geo, Coef c, int64_t lr0, int64_t nlr) {\n  const int lane = threadIdx.x & 63;\n  const int64_t N = geo.N;\n  const int64_t iy = (int64_t(blockIdx.x) * BLOCK + threadIdx.x) * 2;\n  const bool hw = iy > 0, he = iy + 2 < N;\n  for (int64_t p = blockIdx.y; 2 * p < nlr; p += gridDim.y) {\n    const int64_t lr = lr0 + 2 * p;\n    const bool two = 2 * p + 1 < nlr;\n    const int64_t li = lr * N + iy;\n    const d2 vn = *reinterpret_cast<const d2*>(v + li - N);\n    const d2 vc = *reinterpret_cast<const d2*>(v + li);\n    const d2 vs = *reinterpret_cast<const d2*>(v + li + N);\n    const d2 vss = *reinterpret_cast<const d2*>(v + li + 2 * N);     // row lr + 2 <= the last ghost row\n    const d2 u0 = *reinterpret_cast<const d2*>(u + li);\n    const d2 u1 = *reinterpret_cast<const d2*>(u + li + N);\n    double vw0 = __shfl_up(vc.y, 1), ve0 = __shfl_down(vc.x, 1);\n    double vw1 = __shfl_up(vs.y, 1), ve1 = __shfl_down(vs.x, 1);\n    if (lane == 0) {\n      vw0 = hw ? v[li - 1] : 0.0;\n      vw1 = hw ? v[li + N - 1] : 0.0;\n    }\n    if (lane == 63) {\n      ve0 = he ? v[li + 2] : 0.0;\n      ve1 = he ? v[li + N + 2] : 0.0;\n    }\n    d2 o0, o1;\n    o0.x = jvp_pt(c, jdiag(c, u0.x), vn.x, vw0, hw, vc.x, vc.y, true, vs.x);\n    o0.y = jvp_pt(c, jdiag(c, u0.y), vn.y, vc.x, true, vc.y, ve0, he, vs.y);\n    *reinterpret_cast<d2*>(out + li) = o0;\n    if (two) {\n      o1.x = jvp_pt(c, jdiag(c, u1.x), vc.x, vw1, hw, vs.x, vs.y, true, vss.x);\n      o1.y = jvp_pt(c, jdiag(c, u1.y), vc.y, vs.x, true, vs.y, ve1, he, vss.y);\n      *reinterpret_cast<d2*>(out + li + N) = o1;\n    }\n  }\n}\n\ntemplate <int VEC>\n__global__ __launch_bounds__(BLOCK) void k_forward('), ('  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);\n  TimedLaunch tl(ctx, GNK_TIMER_JVP, 24.0 * double(ctx->geo.nrows) * double(ctx->geo.N));\n  DISPATCH_VEC(ctx, k_jvp, L, 0, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr, 0);', '  RowLaunch L = rows(ctx, G, ctx->geo.nrows, vec_of(ctx), 1 << 30);\n  TimedLaunch tl(ctx, GNK_TIMER_JVP, 24.0 * double(ctx->geo.nrows) * double(ctx->geo.N));\n  if (ctx->geo.N % 128 == 0) {\n    L.grid.y = unsigned(std::min<int64_t>((L.nlr + 1) / 2, 65535));\n    hipLaunchKernelGGL(k_jvp2, L.grid, dim3(BLOCK), 0, ctx->stream, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr);\n  } else\n  DISPATCH_VEC(ctx, k_jvp, L, 0, u, v, out, ctx->geo, ctx->coef, L.lr0, L.nlr, 0);')],
    # k_gemv_vjpg: one point per lane (8-B loads; half the V registers -> more waves per SIMD)
    "tv1": [("""  const void* fn = vec_of(ctx) == 2 ? (pend ? vjpg_pick<2, true>(kct) : vjpg_pick<2, false>(kct))
                                    : (pend ? vjpg_pick<1, true>(kct) : vjpg_pick<1, false>(kct));
  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), resident_blocks(ctx, fn));""",
             """  const void* fn = (pend ? vjpg_pick<1, true>(kct) : vjpg_pick<1, false>(kct));
  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, 1, resident_blocks(ctx, fn));""")],
    # k_gemv_vjpg: non-temporal loads of the basis rows
    "tntl": [("      vv[j] = *reinterpret_cast<const d2*>(rowj + boff);",
              "      vv[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(rowj + boff));")],
    # k_gemv_vjpg: non-temporal stores of w, x, g
    "tnts": [("      *reinterpret_cast<d2*>(wcol + li) = ww;", "      __builtin_nontemporal_store(ww, reinterpret_cast<d2*>(wcol + li));"),
             ("    *reinterpret_cast<d2*>(x + li) = xs;\n    if (owned) {\n      const d2 rc", "    __builtin_nontemporal_store(xs, reinterpret_cast<d2*>(x + li));\n    if (owned) {\n      const d2 rc"),
             ("      *reinterpret_cast<d2*>(g + li) = d2{g0, g1};", "      __builtin_nontemporal_store(d2{g0, g1}, reinterpret_cast<d2*>(g + li));")],
    # k_gemv_vjpg: non-temporal V loads and w / x / g stores
    "tnt2": None,
    # k_forward2: non-temporal stores of r
    "fnt": [("    *reinterpret_cast<d2*>(out + li) = f;", "    __builtin_nontemporal_store(f, reinterpret_cast<d2*>(out + li));"),
            ("      *reinterpret_cast<d2*>(out + li + N) = f;", "      __builtin_nontemporal_store(f, reinterpret_cast<d2*>(out + li + N));")],
    # NT stores of the other GNK versions' streaming writes: k_vjp_gemv_t (g), k_cgs (g), k_gemv (x)
    "nt3": [("    if (blockIdx.z == 0) *reinterpret_cast<d2*>(g + li) = d2{g0, g1};", "    if (blockIdx.z == 0) st_nt(g + li, d2{g0, g1});"),
            ("    gg.y = gg.y - s.y;\n    *reinterpret_cast<d2*>(g + li) = gg;", "    gg.y = gg.y - s.y;\n    st_nt(g + li, gg);"),
            ("      acc.y = acc.y + vv.y * cj;\n    }\n    *reinterpret_cast<d2*>(x + li) = acc;", "      acc.y = acc.y + vv.y * cj;\n    }\n    st_nt(x + li, acc);")],
    # k_gemv_vjpg: one point per lane with the NT basis loads of the product's two-point path
    "tv1nt": [("""  const void* fn = vec_of(ctx) == 2 ? (pend ? vjpg_pick<2, true>(kct) : vjpg_pick<2, false>(kct))
                                    : (pend ? vjpg_pick<1, true>(kct) : vjpg_pick<1, false>(kct));
  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), resident_blocks(ctx, fn));""",
             """  const void* fn = (pend ? vjpg_pick<1, true>(kct) : vjpg_pick<1, false>(kct));
  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, 1, resident_blocks(ctx, fn));"""),
              ("      for (int j = 0; j < KCT; ++j) vv[j] = V[min(j, jmax) * ldv + i];",
               "      for (int j = 0; j < KCT; ++j) vv[j] = __builtin_nontemporal_load(V + min(j, jmax) * ldv + i);")],
    # k_gram_v / k_gram_v1: non-temporal loads of the marching south rows (each basis value leaves HBM once)
    "gvnt": [("        vs[j] = *reinterpret_cast<const d2*>(cp + N);\n        eo[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;     // only the strip's edge lanes load",
              "        vs[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(cp + N));\n        eo[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;     // only the strip's edge lanes load"),
             ("        vs[j] = cp[N];\n        eo[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;     // only the strip's edge lanes load",
              "        vs[j] = __builtin_nontemporal_load(cp + N);\n        eo[j] = (edge_w || edge_e) ? cp[eoff] : 0.0;     // only the strip's edge lanes load")],
    # k_gemv_vjpg: one workgroup per row segment (as k_jvp2) instead of the resident persistent grid
    "vjpgrow": [('  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), resident_blocks(ctx, fn));', '  RowLaunch L = rows(ctx, 0, ctx->geo.nrows + 2 * G, vec_of(ctx), 1 << 30);')],
}
VARIANTS["tnt2"] = VARIANTS["tntl"] + VARIANTS["tnts"]


def build(name):
    src = open(SRC).read()
    for old, new in VARIANTS[name]:
        if old not in src:
            raise SystemExit(f"variant {name}: substitution not found: {old[:60]!r}")
        src = src.replace(old, new)
    src = src.replace('#include "../../include/gnk.h"', '#include "gnk.h"')
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, f"gnk_{name}.hip")
    open(path, "w").write(src)
    inc = os.path.join(ROOT, "include")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-w", f"-I{inc}", "-o", os.path.join(OUT, f"libgnk_{name}.so"), path]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return name, r.returncode, r.stderr[-2000:]


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with ThreadPoolExecutor(max_workers=4) as ex:
        for name, rc, err in ex.map(build, names):
            print(name, "ok" if rc == 0 else f"FAILED\n{err}")
