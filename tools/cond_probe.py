"""Per-step conditioning of the projected LS problem on the bench workload.

python tools/cond_probe.py [--grid N] [--steps S]
Prints, per GNK step: basis size k, Gram passes, cond(R_Y) of each pass, cond(R) of the
final factor (= cond(J V)), so the preconditioning policy of lls.py can be checked
against the real workload.
"""
import argparse
import contextlib
import io
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import SingleRankOperator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=41)
    ap.add_argument("--version", default="res_old")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    N = a.grid
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    u_true = prob.u_true
    np.random.seed(42)
    u0 = u_true + 0.1 * np.random.normal(loc=0, scale=1, size=len(u_true))
    dev = torch.device("cuda", 0)
    y = SingleRankOperator(prob, dev).forward(u_true)
    s = gnk.GNKSolver(prob, y, krylow_restart=20, tol=1e-8, max_iter=10 ** 9, version=a.version, device=dev)
    s.setup(u0)
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(a.steps):
            R = None
            if s.step():
                break
            k, npass, conds = s.lls.history[-1]
            R = s.lls.R_last
            print(json.dumps({"k": k, "passes": npass, "cond_RY": [float(c) for c in conds],
                              "cond_R": float(np.linalg.cond(R)), "t": s.trace[-1]["t"]}), file=sys.stderr)


if __name__ == "__main__":
    main()
