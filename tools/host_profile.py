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
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    N = a.grid
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    comm = Comm(single=True)
    stage = BratuDevice(prob, comm)
    u0, y, _ = slab_inputs(stage)
    s = gnk.GNKSolver(prob, y, krylow_restart=20, tol=1e-8, max_iter=10 ** 9, comm=comm, backend=stage.backend)
    s.setup(u0)
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(25):                       # a whole restart cycle: every kernel variant loaded
            s.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(a.steps):
            s.step()
    torch.cuda.synchronize()
    print(f"without profiler: {1e3 * (time.perf_counter() - t0) / a.steps:.3f} ms/step")
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
