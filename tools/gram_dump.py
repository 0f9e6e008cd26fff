"""Dump the Gram of [J V P^-1 | r] (gnk_gram, kbench's gram2 inputs) for several basis sizes k, and time it:
A/B of two builds of libgnk.so for bit-identity and speed (load the other with GNK_LIB=...).

  python tools/gram_dump.py OUTDIR TAG k1,k2,... [--grid N] [--reps R] [--tune key=value,...]
writes OUTDIR/G_TAG_k.npy and prints one JSON line per k (median ms).  Compare two tags with
  python tools/gram_dump.py --compare OUTDIR TAG_A TAG_B
"""
import argparse
import glob
import json
import os
import sys

import numpy as np


def dump(a):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gauss_newton_via_generalized_krylov_subspaces_amd import BratuPdeProblem
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
    torch.cuda.set_device(0)
    N = a.grid
    n = N * N
    dev = BratuDevice(BratuPdeProblem(N + 1, 5, 10), Comm(single=True))
    be, sl = dev.backend, dev.slab
    for kv in filter(None, a.tune.split(",")):
        key, val = kv.split("=")
        be.set_tuning(key, int(val))
    ks = [int(k) for k in a.ks.split(",")]
    kmax = max(ks)
    g = torch.Generator(device=be.device).manual_seed(0)
    V = be.zeros(kmax + 1, sl.length)
    V[:, sl.own] = torch.randn(kmax + 1, n, generator=g, device=be.device, dtype=torch.float64) / np.sqrt(n)
    u, r = dev.vec(), dev.vec()
    u[sl.own] = 0.1 * torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    r[sl.own] = torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
    os.makedirs(a.out, exist_ok=True)
    for k in ks:
        kp = be.gram_dim(k, True)
        rinv = np.zeros((kp, kp))
        rinv[:k + 1, :k + 1] = np.triu(np.ones((k + 1, k + 1))) * 0.1 + np.eye(k + 1)
        rinv_d = be.to_device(rinv.reshape(-1))
        G = be.zeros(kp * kp)
        be.gram(u, V, k, rinv_d, r, G)
        torch.cuda.synchronize()
        ms = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            be.gram(u, V, k, rinv_d, r, G)
            e.record()
            torch.cuda.synchronize()
            ms.append(s.elapsed_time(e))
        np.save(os.path.join(a.out, f"G_{a.tag}_k{k}.npy"), G.cpu().numpy())
        print(json.dumps({"tag": a.tag, "k": k, "grid": N, "ms": float(np.median(ms)),
                          "GBs": 8.0 * n * (k + 2) / (np.median(ms) * 1e-3) / 1e9}), flush=True)


def compare(out, ta, tb):
    for fa in sorted(glob.glob(os.path.join(out, f"G_{ta}_k*.npy"))):
        k = fa.rsplit("_k", 1)[1][:-4]
        fb = os.path.join(out, f"G_{tb}_k{k}.npy")
        A, B = np.load(fa), np.load(fb)
        print(json.dumps({"k": int(k), "bit_identical": bool(np.array_equal(A, B)),
                          "max_abs_diff": float(np.max(np.abs(A - B)))}))


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(*sys.argv[2:5])
    else:
        ap = argparse.ArgumentParser()
        ap.add_argument("out")
        ap.add_argument("tag")
        ap.add_argument("ks")
        ap.add_argument("--grid", type=int, default=8192)
        ap.add_argument("--reps", type=int, default=5)
        ap.add_argument("--tune", default="", help="gnk_set_tuning overrides, e.g. gram_wide=4")
        dump(ap.parse_args())
