"""Diagnostics of segment reductions of the staged Gram pass (gnk_set_segments): per-partition
Gram values of the same inputs on one GPU, determinism, ring depth.  Prints JSON lines."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm, tree_sum  # noqa: E402


def rank_gram(N, world, rank, inp, k, tune):
    c = Comm(single=True, segments=True)
    c.world, c.rank = world, rank
    dev = BratuDevice(gnk.BratuPdeProblem(N + 1, 5, 10), c)
    be = dev.backend
    for kk, vv in tune.items():
        be.set_tuning(kk, vv)
    u, r = dev.load(inp["u"]), dev.load(inp["r"])
    V = be.zeros(k, dev.slab.length)
    for j in range(k):
        V[j].copy_(dev.load(inp["V"][j]))
    kp = be.gram_dim(k, True)
    T = np.zeros((kp, kp))
    T[:k, :k] = np.triu(np.full((k, k), 0.05)) + np.eye(k)
    T[k, k] = 1.0
    G = be.zeros(kp * kp)
    be.gram(u, V, k, be.to_device(T.reshape(-1)), r, G)
    out = G.cpu().numpy().copy()
    be.gram(u, V, k, be.to_device(T.reshape(-1)), r, G)
    again = G.cpu().numpy().copy()
    return out, bool(np.array_equal(out, again))


def host_gram(N, inp, k):
    """[J V T | r]^T [J V T | r] in fp64 NumPy (pairwise BLAS sums) -- a rounding-level reference."""
    from oracle import gnk_oracle as O
    prob = O.BratuPdeProblem(N + 1, 5, 10)
    J = prob.make_jac()(inp["u"])
    W = np.stack([J @ inp["V"][j] for j in range(k)], axis=1)
    T = np.triu(np.full((k, k), 0.05)) + np.eye(k)
    Y = np.hstack([W @ T, inp["r"][:, None]])
    return Y.T @ Y


def main():
    torch.cuda.set_device(0)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    for N in (1024,):
        rng = np.random.default_rng(3)
        n = N * N
        K = 20
        inp = {"V": rng.standard_normal((K, n)) / np.sqrt(n), "u": 0.3 * rng.standard_normal(n),
               "r": rng.standard_normal(n)}
        for k in (12,):
            Gh = host_gram(N, inp, k)
            kp = (k + 1 + 15) // 16 * 16
            for world in (1, 2, 4, 8):
                parts = [rank_gram(N, world, p, inp, k, {})[0].reshape(kp, kp)[:k + 1, :k + 1] for p in range(world)]
                rk = [float(np.abs(q[k, :] - 0).max()) for q in parts]
                tot = tree_sum(np.stack([q.reshape(-1) for q in parts])).reshape(k + 1, k + 1)
                err = np.abs(tot - Gh) / np.sqrt(np.outer(np.diag(Gh), np.diag(Gh)))
                print(json.dumps({"diag": "vs host", "N": N, "k": k, "world": world,
                                  "max_err_tile": float(err[:k, :k].max()), "max_err_rcol": float(err[k, :].max()),
                                  "rr": float(tot[k, k]), "rr_host": float(Gh[k, k]),
                                  "per_rank_rr": [float(q[k, k]) for q in parts], "rk": rk}), flush=True)
    for N in (1024, 2048):
        rng = np.random.default_rng(3)
        n = N * N
        K = 20
        inp = {"V": rng.standard_normal((K, n)) / np.sqrt(n), "u": 0.3 * rng.standard_normal(n),
               "r": rng.standard_normal(n)}
        for k in (3, 8, 12, 16, 18, 20):
            for tune in ({}, {"gram_ring": 5}):
                vals, det = {}, True
                for world in (1, 2, 4, 8):
                    parts = []
                    for p in range(world):
                        g, d = rank_gram(N, world, p, inp, k, tune)
                        parts.append(g)
                        det &= d
                    vals[world] = tree_sum(np.stack(parts))
                kp = int(round(np.sqrt(vals[1].size)))
                diff, where = {}, {}
                for w in (2, 4, 8):
                    rd = (np.abs(vals[w] - vals[1]) / (np.abs(vals[1]) + 1e-300)).reshape(kp, kp)
                    diff[w] = float(rd.max())
                    where[w] = [[int(i), int(j)] for i, j in zip(*np.nonzero(rd))][:12]
                print(json.dumps({"N": N, "k": k, "tune": tune, "deterministic": det, "rel_diff_vs_1": diff,
                                  "differing_entries": where}), flush=True)


if __name__ == "__main__":
    main()
