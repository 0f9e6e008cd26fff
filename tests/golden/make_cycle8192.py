"""One whole restart cycle of the headline workload (8192^2, restart 20, res_old: iterations 1..21,
k = 1..20 and the restart) from the PINNED ORACLE -- the reference itself does not fit the build
container at k = 20 (its hstack / J @ V / QR copies peak above 60 GB; make_golden_large.py's
head8192 fixture stops at k = 4).

This is oracle/gnk_oracle.gauss_newton_krylow (ref:gauss_newton_krylow.py:39-145) with the same
arithmetic in lean memory:
  * the basis is one preallocated C-order (n, kmax) array; V[:, :k] views replace hstack
    (ref:krylow.py:72-73; the same values, gemv with a leading dimension);
  * A = -1 * (J @ V) (ref:gauss_newton_krylow.py:86-89) is written column by column into an F-order
    array (negation is exact) and factorised in place by scipy.linalg.qr(overwrite_a=True), the same
    LAPACK geqrf/orgqr calls with the same workspace queries as the reference's copy;
  * J V is kept (F-order) for Armijo's jdd = sum((J V d)^2) (ref:armijo_goldstein.py:50).
V and J V are file-backed (numpy memmaps under CYCLE_SCRATCH: the page cache holds them, so the
process's anonymous memory stays ~ 25 GB -- at k = 17 an all-anonymous run reached 62 GB).  Variants (each a list of per-iteration ||x_k||, ||r_k||, nfev):
  base      the oracle's arithmetic (numpy dot products, LAPACK Householder QR);
  exact_k1  the one-column steps (k = 1) with exactly rounded sums (math.fsum) -- the cancellation-
            limited step the device's compensated k = 1 path computes (tests/golden/make_sensitivity.py).
The GPU test (tests/test_gpu_baseline_sizes.py) asserts base within max(1e-10, |exact_k1 - base|,
the head8192 envelope), and the bookkeeping exactly.

Usage:  python tests/golden/make_cycle8192.py [base|exact_k1 ...]   (merges into large_cycle8192.json)
"""
import contextlib
import io
import json
import math
import os
import sys
import time

import numpy as np
import scipy
import scipy.linalg
from threadpoolctl import threadpool_limits

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import gnk_oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "large_cycle8192.json")
N = 8192
RESTART = 20
MAX_ITER = 22          # iterations 1..21: k = 1..20, the restart after iteration 20, k = 1 again
THREADS = 8


SCRATCH = os.environ.get("CYCLE_SCRATCH", "/tmp")     # file-backed buffers (page cache, not anonymous RSS)


def _mm(name, shape, order):
    return np.lib.format.open_memmap(os.path.join(SCRATCH, f"cycle8192_{name}.npy"), mode="w+", dtype=np.float64,
                                     shape=shape, fortran_order=(order == "F"))


class LeanBasis:
    """ref:krylow.py:16-73 over a preallocated C-order buffer (file-backed)."""

    def __init__(self, n, kmax):
        self.buf = _mm("V", (n, kmax), "C")
        self.k = 0

    @property
    def basis(self):
        return self.buf[:, :self.k]

    def start(self, x0):
        if np.allclose(x0, np.zeros_like(x0)):
            raise ValueError("x0 is not allowed to be 0 in the gauss_newton_krylow algorithm")
        nrm = np.linalg.norm(x0)
        self.buf[:, 0] = x0 / nrm
        self.k = 1
        return np.array([nrm])

    def x(self, c):
        return self.basis @ c

    def update(self, jac_ev, res_ev):
        if self.buf.shape[0] == self.k:
            raise O.GeneralizedKrylowSubspaceSpansEntireSpace
        g = -(jac_ev.T @ res_ev)
        g = g - self.basis @ (self.basis.T @ g)
        if np.allclose(g, 0, atol=1e-8, rtol=0):
            raise O.GeneralizedKrylowSubspaceBreakdown("breakdown")
        g = g / np.linalg.norm(g)
        self.buf[:, self.k] = g
        self.k += 1


def lls_inplace(A, y, exact_k1):
    """ref:gauss_newton_krylow.py:16-36 on an F-order A that may be overwritten."""
    if exact_k1 and A.shape[1] == 1:
        a = A[:, 0]
        return np.array([math.fsum(a * y) / math.fsum(a * a)])
    q, r = scipy.linalg.qr(A, mode="economic", overwrite_a=True)
    for r_kk in np.diagonal(r):
        if np.isclose(r_kk, 0, atol=1e-8):
            print("A is rank deficient")
    return scipy.linalg.solve_triangular(r, q.T @ y)


class _JVd:
    def __init__(self, JV):
        self.JV = JV

    def __matmul__(self, d):
        return self.JV @ d


def run(variant):
    exact_k1 = variant == "exact_k1"
    prob, y, u0 = O.bratu_workload(N)
    res = prob.make_res(y)
    jac = prob.make_jac()
    n = N * N
    kmax = RESTART + 1
    kr = LeanBasis(n, kmax)
    JVbuf = _mm("JV", (n, kmax), "F")
    Abuf = np.empty((n, kmax), order="F")
    rec = {"xnorm": [], "rnorm": [], "nfev": [], "k": []}
    t0 = time.time()
    c = kr.start(u0)
    res_new = res(kr.x(c))
    nfev = 1
    J = jac(u0)
    for it in range(1, MAX_ITER):
        k = kr.k
        JV, A = JVbuf[:, :k], Abuf[:, :k]
        for j in range(k):
            JV[:, j] = J @ kr.buf[:, j]
            np.multiply(JV[:, j], -1, out=A[:, j])
        r_old = res_new
        d = lls_inplace(A, r_old, exact_k1)
        t, res_new, dn = O.armijo_goldstein(lambda cc: res(kr.x(cc)), c, r_old, _JVd(JV), (), d)
        nfev += dn
        s = np.sum(c ** 2)
        c += t * d
        x = kr.x(c)
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(res(x))))
        rec["nfev"].append(int(nfev))
        rec["k"].append(int(k))
        print(f"  {variant} it {it} k {k} nfev {nfev} ||x|| {rec['xnorm'][-1]!r} ({time.time() - t0:.0f} s)",
              file=sys.stderr, flush=True)
        if t ** 2 * np.sum(d ** 2) <= 1e-8 ** 2 * s:
            raise RuntimeError("converged inside the cycle: not the bench trajectory")
        J = jac(x)
        try:
            kr.update(J, r_old)                                   # version res_old
            c = np.append(c, 0)
        except O.GeneralizedKrylowSubspaceBreakdown:
            print(f"Generalized krylow subspace breakdown at iteration = {it}, basis.shape = {kr.basis.shape}")
        if it % RESTART == 0:
            c = kr.start(kr.x(c))
    rec["seconds"] = time.time() - t0
    return rec


if __name__ == "__main__":
    meta = json.load(open(OUT)) if os.path.exists(OUT) else {
        "generator": "tests/golden/make_cycle8192.py (pinned oracle, lean memory; the reference does not fit "
                     "the build container at k = 20)",
        "numpy": np.__version__, "scipy": scipy.__version__, "openblas_threads": THREADS, "N": N,
        "kwargs": {"krylow_restart": RESTART, "max_iter": MAX_ITER, "version": "res_old"}, "variants": {}}
    for v in sys.argv[1:] or ["base", "exact_k1"]:
        buf = io.StringIO()
        with threadpool_limits(limits=THREADS, user_api="blas"), contextlib.redirect_stdout(buf):
            rec = run(v)
        rec["stdout"] = buf.getvalue().splitlines()
        meta["variants"][v] = rec
        with open(OUT, "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        print("wrote", v, file=sys.stderr)
