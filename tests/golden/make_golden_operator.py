"""Golden fixtures for OPERATOR Jacobians, made by running the REFERENCE (build container only).

The reference uses ``jac_ev`` only through ``@`` and ``.T @`` on the GNK path
(ref:gauss_newton_krylow.py:86, ref:krylow.py:62, ref:armijo_goldstein.py:50), so a
``scipy.sparse.linalg.LinearOperator`` Jacobian runs there.  This script runs the reference's
Rosenbrock chain (p = 1000, the F5 starts of ref:rosenbrock_test.py:20-22, :70, :93-94) with
``jac = aslinearoperator(rosenbrock_problem.jac(x))`` and records, per case, what the reference
does with it:

  * gauss_newton_krylow, all four versions: per-iteration ||x_k||, ||r_k||, nfev, the stdout lines,
    the result's counters -- and whether every one of them equals the sparse-Jacobian run
    (``same_as_sparse``: the LinearOperator products are the same csr/csc kernels, so they do);
  * gauss_newton: the exception the reference raises (its ``is_sparse`` test is False for an
    operator, and ``scipy.linalg.lstsq`` cannot take one, ref:gauss_newton.py:109-116).

Outputs numbers and strings only (tests/golden/operator.json); no reference source travels.

Usage:  OPENBLAS_NUM_THREADS=1 PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_operator.py
"""
import contextlib
import io
import json
import os
import sys

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
sys.dont_write_bytecode = True
REF = os.environ.get("GNK_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import scipy  # noqa: E402
from scipy.sparse.linalg import aslinearoperator  # noqa: E402

import armijo_goldstein as ref_ag  # noqa: E402
import gauss_newton as ref_gn  # noqa: E402
import gauss_newton_krylow as ref_gnk  # noqa: E402
import rosenbrock_problem as ref_rosen  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def run(method, res, x0, jac, **kw):
    rec = {"xnorm": [], "rnorm": [], "nfev": [], "cg_iter": []}

    def cb(x, nfev, cg_iter):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(res(x))))
        rec["nfev"].append(int(nfev))
        rec["cg_iter"].append(None if cg_iter is None else int(cg_iter))

    buf = io.StringIO()
    out = {"exception": None}
    with contextlib.redirect_stdout(buf):
        try:
            r = method(res, x0, jac, callback=cb, **kw)
            out.update(nit=int(r.nit), nrev=int(r.nrev), njev=int(r.njev), success=bool(r.success),
                       xnorm_final=float(np.linalg.norm(r.x)))
        except ref_ag.StepLengthConvergenceError as e:
            out["exception"] = ["StepLengthConvergenceError", e.message]
        except Exception as e:                      # noqa: BLE001 -- what the reference raises is the fixture
            out["exception"] = [type(e).__name__, str(e)]
    out["per_iter"] = rec
    out["stdout"] = buf.getvalue().splitlines()
    return out


def op_jac(x):
    return aslinearoperator(ref_rosen.jac(x))


ref_rosen.parameter_count = 1000
np.random.seed(42)
x_i = np.ones(1000) + 0.1 * np.random.normal(loc=0, scale=1, size=1000)   # ref:rosenbrock_test.py:20-22
x_ii = 2 * np.ones(1000)
x_iii = 2 * np.ones(1000)
x_iii[2] = 1.99
META = {"generator": "tests/golden/make_golden_operator.py", "numpy": np.__version__, "scipy": scipy.__version__,
        "openblas_threads": os.environ.get("OPENBLAS_NUM_THREADS"), "cases": {}}
for name, x0 in (("i", x_i), ("ii", x_ii), ("iii", x_iii)):
    for version in ("res_old", "res_new", "jac_old_res_old", "jac_old_res_new"):
        a = run(ref_gnk.gauss_newton_krylow, ref_rosen.res, x0.copy(), op_jac, version=version)
        b = run(ref_gnk.gauss_newton_krylow, ref_rosen.res, x0.copy(), ref_rosen.jac, version=version)
        a["same_as_sparse"] = a == b
        META["cases"][f"rosen1000_{name}_{version}_op"] = a
        print(name, version, a.get("nit"), a.get("nrev"), "same_as_sparse", a["same_as_sparse"], flush=True)
    g = run(ref_gn.gauss_newton, ref_rosen.res, x0.copy(), op_jac)
    META["cases"][f"rosen1000_{name}_gn_op"] = g
    print(name, "gn", g["exception"], flush=True)

with open(os.path.join(OUT, "operator.json"), "w") as f:
    json.dump(META, f, indent=1)
