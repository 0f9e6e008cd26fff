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
  cholqr    the device's least-squares arithmetic (lls.CholQR2Solver._passes) instead of Householder:
            the k = 1 step on exactly rounded sums in k_lls's operation order, then for k >= 2 preconditioned CholeskyQR -- P = blockdiag(R_prev, 1),
            Y = (J V) P^-1 (fp64 BLAS), the Gram of [Y | r] in extended precision (x87 80-bit products
            and sums over 64 Ki-row chunks, the chunk sums kept as double-double pairs and added exactly
            by math.fsum: ~1e-19 relative, orders below an fp64 Gram), the new column rescaled by
            sqrt(G_kk), another pass with P = R_Y P while cond(R_Y) > 30, R = R_Y P, d = -R^-1 R_Y^-T Y^T r,
            and Armijo's jdd = ||R d||^2 (the device's).  Everything else -- the basis update, the
            trials -- is the base arithmetic, so |cholqr - base| is the move of the reference's
            trajectory under an equally valid factorisation, and |device - cholqr| what is left.
The GPU test (tests/test_gpu_baseline_sizes.py) asserts base within max(1e-10, |exact_k1 - base|,
the head8192 envelope), and the bookkeeping exactly.

Usage:  python tests/golden/make_cycle8192.py [base|exact_k1|cholqr ...]   (merges into large_cycle8192.json)
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


def _gram_ext(Y, r):
    """[Y | r]^T [Y | r] (F-order Y, n x k) with x87 80-bit products / sums per 64 Ki-row chunk, the
    chunk sums split into double-double (hi, lo) and summed exactly (math.fsum), rounded once."""
    n, k = Y.shape
    CH = 1 << 16
    m = k + 1
    parts = [[[] for _ in range(m)] for _ in range(m)]
    Z = np.empty((CH, m), dtype=np.longdouble, order="F")
    for lo in range(0, n, CH):
        hi = min(n, lo + CH)
        L = hi - lo
        for j in range(k):
            Z[:L, j] = Y[lo:hi, j]
        Z[:L, k] = r[lo:hi]
        for i in range(m):
            zi = Z[:L, i]
            for j in range(i, m):
                sv = np.dot(zi, Z[:L, j])
                h = float(sv)
                parts[i][j] += [h, float(sv - np.longdouble(h))]
    G = np.empty((m, m))
    for i in range(m):
        for j in range(i, m):
            G[i, j] = G[j, i] = math.fsum(parts[i][j])
    return G


class CholQRLS:
    """lls.CholQR2Solver._passes (host form) on the fp64 J V of the reference basis."""
    COND_ACCEPT = 30.0

    def __init__(self):
        self.R_prev = None
        self.passes = []

    def restart(self):
        self.R_prev = None

    def solve(self, JV, Ybuf, r):
        import scipy.linalg as sl
        k = JV.shape[1]
        if k == 1 or self.R_prev is None:
            a = JV[:, 0] if k == 1 else None
            if k != 1:
                raise RuntimeError("no preconditioner at k > 1: not the bench trajectory")
            # the k = 1 step on exactly rounded sums G = [||Jv||^2, Jv.r], in k_lls's arithmetic: the pass's
            # rescale divides the Gram's row and column by s = sqrt(g00) (g00 / s / s, not exactly 1), then
            # Cholesky ry = sqrt(.), z = (g01 / s) / ry, R = ry s, d = -(z / R)
            g00 = math.fsum(a * a)
            g01 = math.fsum(a * r)
            s = math.sqrt(g00)
            ry = math.sqrt((g00 / s) / s)
            z = (g01 / s) / ry
            R = np.array([[ry * s]])
            d = np.array([-(z / R[0, 0])])
            self.R_prev = R
            self.passes.append((k, 1, [1.0]))
            return d, R
        P = np.zeros((k, k))
        P[:k - 1, :k - 1] = self.R_prev
        P[k - 1, k - 1] = 1.0
        conds = []
        for it in range(4):
            T = sl.solve_triangular(P, np.eye(k), lower=False)
            Y = Ybuf[:, :k]
            np.matmul(JV, T, out=Y)
            G = _gram_ext(Y, r)
            if it == 0:
                s = math.sqrt(G[k - 1, k - 1])
                G[k - 1, :] /= s
                G[:, k - 1] /= s
                P[k - 1, k - 1] = s
            Ry = sl.cholesky(G[:k, :k], lower=False)
            sv = np.linalg.svd(Ry, compute_uv=False)
            conds.append(float(sv[0] / sv[-1]))
            if conds[-1] <= self.COND_ACCEPT or it == 3:
                z = sl.solve_triangular(Ry, G[:k, k], trans="T", lower=False)
                R = Ry @ P
                break
            P = Ry @ P
        d = -sl.solve_triangular(R, z, lower=False)
        self.R_prev = R                       # the next step's preconditioner (blockdiag(R, scale))
        self.passes.append((k, len(conds), conds))
        return d, R


class _Rd:
    """Armijo's jac_ev @ d with the device's jdd = ||R d||^2 (lls.py)."""

    def __init__(self, R):
        self.R = R

    def __matmul__(self, d):
        return self.R @ d


class _JVd:
    def __init__(self, JV):
        self.JV = JV

    def __matmul__(self, d):
        return self.JV @ d


def run(variant):
    exact_k1 = variant == "exact_k1"
    chol = CholQRLS() if variant == "cholqr" else None
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
            if chol is None:
                np.multiply(JV[:, j], -1, out=A[:, j])
        r_old = res_new
        if chol is None:
            d = lls_inplace(A, r_old, exact_k1)
            jv = _JVd(JV)
        else:
            d, R = chol.solve(JV, Abuf, r_old)
            jv = _Rd(R)
        t, res_new, dn = O.armijo_goldstein(lambda cc: res(kr.x(cc)), c, r_old, jv, (), d)
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
            if chol is not None:
                chol.restart()
    rec["seconds"] = time.time() - t0
    if chol is not None:
        rec["ls_passes"] = chol.passes
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
