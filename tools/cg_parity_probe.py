"""Measure the GPU CG paths against the golden reference runs (cg_iter per outer iteration, iterate
distances) -- informs the tolerances in tests/tolerances.py.  Prints one JSON line."""
import contextlib
import io
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from oracle import gnk_oracle as O  # noqa: E402

meta = json.load(open("tests/golden/golden.json"))
arr = dict(np.load("tests/golden/golden.npz"))
out = {}
prob = gnk.BratuPdeProblem(101, 5, 10)
y = O.BratuPdeProblem(101, 5, 10).pde_operator(O.BratuPdeProblem(101, 5, 10).u_true)
for name, kw in [("bratu100_gn", {})]:
    rec = []
    with contextlib.redirect_stdout(io.StringIO()):
        r = gnk.gauss_newton(prob.make_res(y), arr["bratu100_u0"], prob.make_jac(),
                             callback=lambda x, nfev, cg_iter: rec.append((np.linalg.norm(x), cg_iter)), **kw)
    ref = meta["cases"][name]["per_iter"]
    out[name] = {"cg_iter": [c for _, c in rec], "ref": ref["cg_iter"],
                 "max_rel_x": float(np.max(np.abs(np.array([x for x, _ in rec]) - ref["xnorm"]) / np.array(ref["xnorm"])))}
for N in (24, 100):
    p2, y2, u2 = O.bratu_workload(N)
    r0 = p2.make_res(y2)(u2)
    dp = gnk.BratuPdeProblem(N + 1, 5, 10)
    for pre, rtol in [(False, 1e-4), (True, 1e-4), (True, 1e-8)]:
        name = f"cgls{N}_pre{int(pre)}" + ("_rtol1e-8" if rtol == 1e-8 else "")
        x, it = gnk.cg_least_squares(-1 * dp.make_jac()(u2), r0, cg_rtol=rtol, preconditioner=pre)
        xr = arr[name + "__x"]
        out[name] = {"it": it, "ref": meta["cases"][name]["cg_iter"], "max_abs_over_scale": float(np.abs(x - xr).max() / np.abs(xr).max())}
for p in (2, 1000):
    res, jac = O.rosenbrock(p)
    from tests.test_generic_host import rosen_x0
    for x0n in (["m1_1", "2_2"] if p == 2 else ["i", "ii", "iii"]):
        rec = []
        with contextlib.redirect_stdout(io.StringIO()):
            gnk.gauss_newton(res, rosen_x0(arr, p, x0n), jac, callback=lambda x, nfev, cg_iter: rec.append((np.linalg.norm(x), cg_iter)))
        ref = meta["cases"][f"rosen{p}_{x0n}_gn"]["per_iter"]
        n = min(len(rec), len(ref["xnorm"]))
        out[f"rosen{p}_{x0n}_gn"] = {"cg_equal": [c for _, c in rec] == ref["cg_iter"], "cg": [c for _, c in rec][:25], "ref": ref["cg_iter"][:25], "cg": [c for _, c in rec][:25], "ref": ref["cg_iter"][:25],
                                     "max_rel_x": float(np.max(np.abs(np.array([x for x, _ in rec[:n]]) - ref["xnorm"][:n]) / np.array(ref["xnorm"][:n])))}
print(json.dumps(out))
