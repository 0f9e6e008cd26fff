"""cProfile of the GNK step loop on the bench workload (host overhead per outer iteration).

python tools/host_profile.py [--grid N] [--steps S]
"""
import argparse
import contextlib
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import SingleRankOperator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    N = a.grid
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    np.random.seed(42)
    u0 = prob.u_true + 0.1 * np.random.normal(loc=0, scale=1, size=N * N)
    dev = torch.device("cuda", 0)
    y = SingleRankOperator(prob, dev).forward(prob.u_true)
    s = gnk.GNKSolver(prob, y, krylow_restart=20, tol=1e-8, max_iter=10 ** 9, device=dev)
    s.setup(u0)
    with contextlib.redirect_stdout(io.StringIO()):
        s.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(a.steps):
            s.step()
    torch.cuda.synchronize()
    pr.disable()
    el = time.perf_counter() - t0
    print(f"{a.steps} steps, {1e3 * el / a.steps:.3f} ms/step")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
