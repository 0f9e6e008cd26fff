"""Interleaved A/B of gnk_set_tuning variants of the Gram pass on one GPU (8192^2, the bench's
preconditioned pass with r): median ms of gnk_gram (kernel + reduction + scatter) per (k, variant).

  python tools/tune_ab.py --ks 8,9,10 --variants "default;gram_v1min=-1;gram_path=1"
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
    ap.add_argument("--ks", default="8,9")
    ap.add_argument("--variants", default="default")
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    N = a.grid
    n = N * N
    ks = [int(x) for x in a.ks.split(",")]
    dev = BratuDevice(BratuPdeProblem(N + 1, 5, 10), Comm(single=True))
    be, sl = dev.backend, dev.slab
    g = torch.Generator(device=be.device).manual_seed(0)
    K = max(ks)
    V = be.zeros(K, sl.length)
    V[:, sl.own] = torch.randn(K, n, generator=g, device=be.device, dtype=torch.float64) / np.sqrt(n)
    u, r = dev.vec(), dev.vec()
    u[sl.own] = 0.1 * torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    r[sl.own] = torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    variants = a.variants.split(";")

    def apply(v):
        for key in ("gram_path", "gram_ring", "gram_v1min", "gram_rpr", "gram_wide"):
            be.set_tuning(key, 0)
        if v != "default":
            for kv in v.split(","):
                key, val = kv.split("=")
                be.set_tuning(key, int(val))

    for k in ks:
        kp = be.gram_dim(k, True)
        rinv = np.zeros((kp, kp))
        rinv[:k + 1, :k + 1] = np.triu(np.ones((k + 1, k + 1))) * 0.1 + np.eye(k + 1)
        rinv_d = be.to_device(rinv.reshape(-1))
        G = be.zeros(kp * kp)
        res = {v: [] for v in variants}
        for _ in range(a.reps):
            for v in variants:
                apply(v)
                be.gram(u, V[:k], k, rinv_d, r, G)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                be.gram(u, V[:k], k, rinv_d, r, G)
                e.record()
                torch.cuda.synchronize()
                res[v].append(s.elapsed_time(e))
        apply("default")
        print(json.dumps({"grid": N, "k": k, "ms": {v: float(np.median(x)) for v, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
