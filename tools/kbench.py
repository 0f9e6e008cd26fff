"""Per-kernel microbenchmark on the 8192^2 slab (for rocprofv3 counter passes and A/B tests).

python tools/kbench.py [--grid N] [--k K] [--reps R] [--kernels gram1,gram2,jvp,gemv,vjpg,norm,cgs,resid,cg,gemvp]
Prints one JSON line with the median ms and algorithmic GB/s per kernel.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gauss_newton_via_generalized_krylov_subspaces_amd import BratuPdeProblem  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=8192)
    ap.add_argument("--k", type=int, default=15)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--kernels", default="gram1,gram2,jvp,gemv,vjpg,cgs,resid,cg")
    ap.add_argument("--tune", default="", help="gnk_set_tuning overrides, e.g. gram_path=1,gram_ring=4")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    N, k = a.grid, a.k
    n = N * N
    dev = BratuDevice(BratuPdeProblem(N + 1, 5, 10), Comm(single=True))
    be, sl = dev.backend, dev.slab
    for kv in filter(None, a.tune.split(",")):
        key, val = kv.split("=")
        be.set_tuning(key, int(val))
    g = torch.Generator(device=be.device).manual_seed(0)
    V = be.zeros(k + 1, sl.length)
    for j in range(k + 1):                   # a column at a time: no (k + 1) x n temporary at 16384^2
        V[j, sl.own] = torch.randn(n, generator=g, device=be.device, dtype=torch.float64) / np.sqrt(n)
    u, r, x, y, t1 = (dev.vec() for _ in range(5))
    u[sl.own] = 0.1 * torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    r[sl.own] = torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    y.copy_(r)
    c = be.to_device(np.random.default_rng(0).standard_normal(k + 1))
    kp = be.gram_dim(k, True)
    G = be.zeros(kp * kp)
    rinv = np.zeros((kp, kp)); rinv[:k + 1, :k + 1] = np.triu(np.ones((k + 1, k + 1))) * 0.1 + np.eye(k + 1)
    rinv_d = be.to_device(rinv.reshape(-1))
    h = be.zeros(k + 1)
    st = be.zeros(2)
    d = dev.vec()
    be.jdiag(u, d)
    q = dev.vec()
    # gram2n (Gram of k + 1 columns), trialp (pending first trial over k columns, the last pending)
    kpn = be.gram_dim(k + 1, True)
    tf = np.zeros((kpn, kpn)); tf[:k + 2, :k + 2] = np.triu(np.ones((k + 2, k + 2))) * 0.1 + np.eye(k + 2)
    tf_d = be.to_device(tf.reshape(-1))
    Gn = be.zeros(kpn * kpn)
    hh = be.to_device(0.01 * np.random.default_rng(1).standard_normal(k))
    ops = {
        "gram1": (lambda: be.gram(u, V, k, None, None, G), 8.0 * n * (k + 1)),
        "gram2": (lambda: be.gram(u, V, k, rinv_d, r, G), 8.0 * n * (k + 2)),
        "jvp": (lambda: be.jvp(u, r, t1), 24.0 * n),
        "gemv": (lambda: be.gemv(V, k, c, x), 8.0 * (sl.length * (k + 1))),
        "vjpg": (lambda: be.vjp_gemv_t(u, r, V, k, V[k], h), 8.0 * n * (k + 4)),
        "norm": (lambda: be.normalize_jnorm(u, r, 3.0, t1, st), 24.0 * n),
        "cgs": (lambda: be.cgs_update(V, k, h, V[k], st), 8.0 * n * (k + 2)),
        "resid": (lambda: be.residual(x, y, t1, st), 24.0 * n),
        "cg": (lambda: be.cg_matvec(d, r, q, st), 24.0 * n),
        "gram2n": (lambda: be.gram(u, V, k + 1, tf_d, r, Gn), 8.0 * n * (k + 3)),
        "trialp": (lambda: be.gemv_vjp_gemv_t_pending(V, k - 1, c, hh, r, x, V[k], h, st), 8.0 * n * (k + 5)),
        # restart point with the pending column settled (k settled columns + the pending one: k + 1 reads, 2 writes)
        "gemvp": (lambda: be.gemv_pending(V, k, c, hh, x, st), 8.0 * n * (k + 3)),
    }
    out = {"grid": N, "k": k}
    for name in a.kernels.split(","):
        fn, by = ops[name]
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            ms.append(s.elapsed_time(e))
        m = float(np.median(ms))
        out[name] = {"ms": m, "GBs": by / m / 1e6}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
