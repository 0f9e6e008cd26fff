"""Time the fused first trial with the pending column (gnk_basis_gemv_vjp_gemv_t_pending) at several basis widths:
    python tools/trial_dump.py TAG kk1,kk2,... [--grid N] [--reps R] [--tune key=value,...]
prints one JSON line per width (median ms, GB/s of the k + 5 vectors it moves)."""
import argparse
import hashlib
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
    ap.add_argument("tag")
    ap.add_argument("kks")
    ap.add_argument("--grid", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tune", default="")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    N = a.grid
    n = N * N
    dev = BratuDevice(BratuPdeProblem(N + 1, 5, 10), Comm(single=True))
    be, sl = dev.backend, dev.slab
    for kv in filter(None, a.tune.split(",")):
        key, val = kv.split("=")
        be.set_tuning(key, int(val))
    kks = [int(k) for k in a.kks.split(",")]
    kmax = max(kks)
    g = torch.Generator(device=be.device).manual_seed(0)
    V = be.zeros(kmax, sl.length)
    V[:, sl.own] = torch.randn(kmax, n, generator=g, device=be.device, dtype=torch.float64) / np.sqrt(n)
    r = dev.vec()
    r[sl.own] = torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    c = be.to_device(np.linspace(0.5, 1.5, kmax))
    hh = be.to_device(np.zeros(kmax))
    x, gg, h, st = dev.vec(), dev.vec(), be.zeros(kmax + 1), be.zeros(4)
    for kk in kks:
        k = kk - 1
        be.gemv_vjp_gemv_t_pending(V, k, c, hh, r, x, gg, h, st)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            be.gemv_vjp_gemv_t_pending(V, k, c, hh, r, x, gg, h, st)
            e.record()
            torch.cuda.synchronize()
            ms.append(s.elapsed_time(e))
        med = float(np.median(ms))
        print(json.dumps({"tag": a.tag, "kk": kk, "grid": N, "ms": med, "GBs": 8.0 * n * (k + 5) / (med * 1e-3) / 1e9,
                          "h0": float(h[0].item()),
                          "bits": hashlib.sha1(b"".join(t.cpu().numpy().tobytes() for t in (h[:kk], x[sl.own], gg[sl.own], st[:2])))
                          .hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
