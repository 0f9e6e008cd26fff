"""A/B of the Gram pass's row decomposition on one GPU (8192^2, the bench's preconditioned pass with r):
the library's rows per range vs the finer, fixed one an 8-rank slab uses (tuning gram_rpr).  Prints one
JSON line per (k, rpr): median ms of gnk_gram (kernel + reduction + scatter) over interleaved reps."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gauss_newton_via_generalized_krylov_subspaces_amd import BratuPdeProblem  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402


def main(N=8192, ks=(3, 6, 7, 8, 9, 10, 12, 16, 17, 20), reps=15):
    torch.cuda.set_device(0)
    n = N * N
    dev = BratuDevice(BratuPdeProblem(N + 1, 5, 10), Comm(single=True))
    be, sl = dev.backend, dev.slab
    g = torch.Generator(device=be.device).manual_seed(0)
    K = max(ks)
    V = be.zeros(K, sl.length)
    V[:, sl.own] = torch.randn(K, n, generator=g, device=be.device, dtype=torch.float64) / np.sqrt(n)
    u, r = dev.vec(), dev.vec()
    u[sl.own] = 0.1 * torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    r[sl.own] = torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    for k in ks:
        base = 32 if k <= 7 else (64 if k <= 9 else 128)
        kp = be.gram_dim(k, True)
        rinv = np.zeros((kp, kp))
        rinv[:k + 1, :k + 1] = np.triu(np.ones((k + 1, k + 1))) * 0.1 + np.eye(k + 1)
        rinv_d = be.to_device(rinv.reshape(-1))
        G = be.zeros(kp * kp)
        res = {}
        variants = (0, base, 2 * base, 4 * base)
        for rp in variants:
            res[rp] = []
        for _ in range(reps):
            for rp in variants:
                be.set_tuning("gram_rpr", rp)
                be.gram(u, V[:k], k, rinv_d, r, G)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                be.gram(u, V[:k], k, rinv_d, r, G)
                e.record()
                torch.cuda.synchronize()
                res[rp].append(s.elapsed_time(e))
        be.set_tuning("gram_rpr", 0)
        line = {"grid": N, "k": k, "ms": {str(rp): float(np.median(v)) for rp, v in res.items()}}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
