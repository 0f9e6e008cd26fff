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
