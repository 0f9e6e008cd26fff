"""Conditioning of J V under structured preconditioners on the oracle's GNK run:
full P = R_prev, column scaling, and P with only its first m rows dense ("rows m") or its leading m x m block
("blk m"), per basis size k.  CPU only (oracle).  python tools/cond_struct.py [N]"""
import contextlib
import io
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gnk_oracle as O
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
prob, y, u0 = O.bratu_workload(N)
orig = O.linear_least_squares
prevR = [None]
def cnd(M):
    s = np.linalg.svd(M, compute_uv=False); return s[0] / s[-1]
def lls(A, yy):
    Z = -A
    k = Z.shape[1]
    q, r = np.linalg.qr(Z)
    if prevR[0] is not None and prevR[0].shape[0] == k - 1 and k >= 6:
        nrm = np.linalg.norm(Z, axis=0)
        P = np.eye(k); P[:k-1,:k-1] = prevR[0]; P[k-1,k-1] = nrm[-1]
        out = [f"k={k:2d} full {cnd(np.linalg.solve(P.T, Z.T).T):.3g}"]
        for m in (1, 2, 3, 4, 6):
            Pa = np.diag(np.diag(P)); Pa[:m,:m] = P[:m,:m]
            Pb = np.diag(np.diag(P)); Pb[:m,:] = P[:m,:]
            out.append(f"m={m}: blk {cnd(np.linalg.solve(Pa.T, Z.T).T):.3g} rows {cnd(np.linalg.solve(Pb.T, Z.T).T):.3g}")
        print(" | ".join(out), flush=True)
    prevR[0] = r
    return orig(A, yy)
O.linear_least_squares = lls
with contextlib.redirect_stderr(io.StringIO()):
    O.gauss_newton_krylow(prob.make_res(y), u0, prob.make_jac(), krylow_restart=20, max_iter=21, version="res_old")
