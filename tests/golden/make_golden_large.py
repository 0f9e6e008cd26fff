"""Golden fixtures at BASELINE.json's sizes, produced by running the REFERENCE itself.

Like make_golden.py this imports the reference (read-only at /root/reference in the build
container) and writes only inputs' recipes and expected outputs -- per-iteration norms,
bookkeeping, stdout, subsampled solution vectors -- to ``tests/golden/large_<case>.json`` /
``.npz``.  The GPU box regenerates the inputs from the same recipe (BratuPdeProblem(N+1, 5, 10),
u0 = u_true + 0.1 N(0,1) with np.random.seed(42), ref:bratu_pde_test.py:22-36) and compares.

Cases (pick with argv[1]):
  c2        N = 1024, krylow_restart = 20, max_iter = 100, res_old and res_new  (BASELINE configs[1];
            ref:gauss_newton_krylow.py:84-136): every iteration's ||x_k||, ||r_k||, nfev, stdout.
  head8192  N = 8192, krylow_restart = 20, res_old, max_iter = 5 (the first 4 outer iterations of
            the bench workload, k = 1..4): per-iteration ||x_k||, ||r_k||, nfev.  RSS ~ 37 GB.
  c3        N = 8192, first Gauss-Newton step's CGLS (ref:gauss_newton.py:50-58: Jacobi, A = -jac(u0),
            y = res(u0)) with rtol 1e-8 capped at CG_CAP iterations (scipy.sparse.linalg.cg with
            maxiter, the reference's own call otherwise): per-iteration ||x_k|| and the true normal-
            equation residual ||A^T y - A^T A x_k||, and x subsampled.

Usage:  OPENBLAS_NUM_THREADS=1 PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_large.py c2
"""
import contextlib
import io
import json
import os
import sys
import time

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
sys.dont_write_bytecode = True
REF = os.environ.get("GNK_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import scipy  # noqa: E402
import scipy.sparse.linalg  # noqa: E402

import armijo_goldstein as ref_ag  # noqa: E402
import bratu_pde_problem as ref_bratu  # noqa: E402
import gauss_newton_krylow as ref_gnk  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SUB = 997          # solution vectors are kept at every SUB-th entry (plus their norm)
CG_CAP = 30


def workload(N):
    prob = ref_bratu.BratuPdeProblem(N + 1, 5, 10)
    y = prob.pde_operator(prob.u_true)
    np.random.seed(42)
    u0 = prob.u_true + 0.1 * np.random.normal(loc=0, scale=1, size=len(prob.u_true))
    return prob, y, u0


def meta_base(case, **kw):
    return {"generator": "tests/golden/make_golden_large.py " + case, "numpy": np.__version__,
            "scipy": scipy.__version__, "openblas_threads": os.environ.get("OPENBLAS_NUM_THREADS"),
            "subsample_stride": SUB, **kw}


def gnk_case(res, u0, jac, **kw):
    rec = {"xnorm": [], "rnorm": [], "nfev": []}
    t0 = time.time()

    def cb(x, nfev, cg_iter):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(res(x))))
        rec["nfev"].append(int(nfev))
        print(f"  it {len(rec['nfev'])} nfev {nfev} ||x|| {rec['xnorm'][-1]!r} ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)

    buf = io.StringIO()
    exc = result = None
    with contextlib.redirect_stdout(buf):
        try:
            result = ref_gnk.gauss_newton_krylow(res, u0, jac, callback=cb, **kw)
        except ref_ag.StepLengthConvergenceError as e:
            exc = ["StepLengthConvergenceError", e.message]
    out = {"per_iter": rec, "stdout": buf.getvalue().splitlines(), "exception": exc, "kwargs": kw,
           "seconds": time.time() - t0}
    arrays = {}
    if result is not None:
        out.update(success=bool(result.success), nrev=int(result.nrev), njev=int(result.njev), nit=int(result.nit),
                   xnorm_final=float(np.linalg.norm(result.x)))
        arrays["x_sub"] = result.x[::SUB].copy()
    return out, arrays


def write(name, meta, arrays):
    with open(os.path.join(OUT, f"large_{name}.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    if arrays:
        np.savez_compressed(os.path.join(OUT, f"large_{name}.npz"), **arrays)
    print("wrote", name)


def case_c2():
    prob, y, u0 = workload(1024)
    meta = meta_base("c2", N=1024, cases={})
    arrays = {}
    for version in ("res_old", "res_new"):
        print("c2", version, flush=True)
        out, arr = gnk_case(prob.make_res(y), u0, prob.make_jac(), krylow_restart=20, max_iter=100, version=version)
        meta["cases"][version] = out
        arrays.update({f"{version}__{k}": v for k, v in arr.items()})
    write("c2", meta, arrays)


def case_head8192():
    prob, y, u0 = workload(8192)
    meta = meta_base("head8192", N=8192, cases={})
    out, arr = gnk_case(prob.make_res(y), u0, prob.make_jac(), krylow_restart=20, max_iter=5, version="res_old")
    meta["cases"]["res_old"] = out
    write("head8192", meta, {f"res_old__{k}": v for k, v in arr.items()})


def case_c3():
    prob, y, u0 = workload(8192)
    t0 = time.time()
    res = prob.make_res(y)
    r0 = res(u0)
    A = -1 * prob.make_jac()(u0)
    del prob
    p = A.shape[1]
    ATA = scipy.sparse.linalg.LinearOperator((p, p), matvec=lambda x: A.T @ (A @ x))
    b = A.T @ r0
    dinv = 1 / (A.T @ A).diagonal()                     # ref:gauss_newton.py:50-54
    M = scipy.sparse.diags(dinv)
    rec = {"xnorm": [], "resnorm": []}

    def cb(x):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["resnorm"].append(float(np.linalg.norm(b - ATA @ x)))
        print(f"  cg {len(rec['xnorm'])} ||x|| {rec['xnorm'][-1]!r} ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)

    x, info = scipy.sparse.linalg.cg(ATA, b, M=M, callback=cb, rtol=1e-8, maxiter=CG_CAP)
    meta = meta_base("c3", N=8192, cg_cap=CG_CAP, rtol=1e-8, info=int(info), bnorm=float(np.linalg.norm(b)),
                     per_iter=rec, xnorm_final=float(np.linalg.norm(x)), seconds=time.time() - t0)
    write("c3", meta, {"x_sub": x[::SUB].copy(), "dinv_sub": dinv[::SUB].copy(), "b_sub": b[::SUB].copy()})


if __name__ == "__main__":
    {"c2": case_c2, "head8192": case_head8192, "c3": case_c3}[sys.argv[1]]()
