"""Ablation / experiment builds of libgnk.so (tooling only: the product source is never edited).

python tools/build_variants.py NAME [NAME ...]      -> tools/_diag/libgnk_NAME.so
Each variant is the product source with the text substitutions listed in VARIANTS applied (every
substitution must match, else the build stops).  Load one with GNK_LIB=tools/_diag/libgnk_NAME.so.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gauss_newton_via_generalized_krylov_subspaces_amd", "csrc", "gnk_kernels.hip")
OUT = os.path.join(ROOT, "tools", "_diag")

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
}


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
