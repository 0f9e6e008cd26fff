"""Rounding-sensitivity envelopes of the REFERENCE trajectories (oracle only; no reference import).

A GPU parity bound looser than north_star's 1e-10 is only accepted where the reference's OWN
arithmetic, reordered in an algebraically equivalent way, moves its trajectory at least that much.
For each case below the oracle (oracle/gnk_oracle.py, the CPU restatement of the reference, pinned by
the golden fixtures) is re-run with such reorderings, each at 1 and at 8 OpenBLAS threads (the
reference's own result depends on the thread count):
  base          the oracle as is (LAPACK Householder QR of -J V);
  exact_k1      the one-column least-squares steps (k = 1: d = (a . r) / (a . a), a cancellation-heavy
                dot product at large N) with exactly rounded sums (math.fsum);
  perm<s>       Householder QR of the row-permuted [A | y] (permutation seed s);
  perm<s>+k1    both;
  cholqr2       the least-squares step by CholeskyQR2 (R from the Cholesky factor of the Gram of A,
                twice; Q^T y = R^-T A^T y) instead of Householder -- the same factorisation in exact
                arithmetic, and the family the device solve belongs to;
  cholqr2b<P>   the same with every Gram summed over P row blocks in order (P = 4, 64, 256: the
                device's per-block partials; multi-slab / short-restart cases);
  slab<P>       every reduction ordered as a P-rank slab run (P = 2..8) orders it: TSQR over P row blocks
                (Householder QR per block, QR of the stacked R factors) and the Krylov update's V^T g,
                ||g|| summed block by block in rank order (multi-slab cases only).
The per-iteration relative distance of every variant from the reference trajectory (the reference's
own fixture where one exists -- tests/golden/golden.json, large_*.json -- else the 1-thread oracle)
is recorded, and ``envelope`` is the per-iteration maximum over all variants.  Where the signed
distances are recorded too (``xs`` / ``rs``), ``diameter`` is the per-iteration spread of the whole
family (the reference included): max - min of the signed distances, i.e. how far two equivalent
roundings of the reference's arithmetic can land from each other -- this build being one more.
tests/tolerances.py turns it into the bound max(1e-10, diameter) (else envelope);
tests/test_oracle_sensitivity.py recomputes the cheap cases live and checks them against this file.

Usage:  python tests/golden/make_sensitivity.py <case> [<case> ...]   (cases: see CASES; "all")
"""
import contextlib
import io
import json
import math
import os
import sys

import numpy as np
import scipy.linalg
from threadpoolctl import threadpool_limits

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import gnk_oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
PATH = os.environ.get("SENS_OUT", os.path.join(OUT, "sensitivity.json"))   # (merge tooling: SENS_OUT)
_LLS = O.linear_least_squares
_UPDATE = O.KrylovBasis.update
_ARMIJO = O.armijo_goldstein
THREADS = (1, 8)


def lls_variant(exact_k1, seed):
    def lls(A, y):
        if exact_k1 and A.shape[1] == 1:
            a = A[:, 0]
            return np.array([math.fsum(a * y) / math.fsum(a * a)])
        if seed is not None:
            p = np.random.default_rng(seed).permutation(A.shape[0])
            return _LLS(np.ascontiguousarray(A[p]), y[p])
        return _LLS(A, y)
    return lls


def cholqr2_lls(A, y):
    """min ||A d - y|| by CholeskyQR2 (prints the reference's rank messages from its R)."""
    R1 = scipy.linalg.cholesky(A.T @ A, lower=False)
    Q1 = scipy.linalg.solve_triangular(R1, A.T, trans="T", lower=False).T
    R2 = scipy.linalg.cholesky(Q1.T @ Q1, lower=False)
    R = R2 @ R1
    for r_kk in np.diagonal(R):
        if np.isclose(r_kk, 0, atol=1e-8):
            print("A is rank deficient")
    z = scipy.linalg.solve_triangular(R, A.T @ y, trans="T", lower=False)
    return scipy.linalg.solve_triangular(R, z)


def cholqr2_blocked(P):
    """CholeskyQR2 with every Gram (A^T A, A^T y) accumulated over P row blocks in order -- the shape of
    the device solve's reduction (per-block partials summed in a fixed order)."""
    def gram(X, Y):
        n = X.shape[0]
        edges = np.linspace(0, n, P + 1).astype(int)
        g = 0.0
        for a, b in zip(edges[:-1], edges[1:]):
            g = g + X[a:b].T @ Y[a:b]
        return g

    def lls(A, y):
        R1 = scipy.linalg.cholesky(gram(A, A), lower=False)
        Q1 = scipy.linalg.solve_triangular(R1, A.T, trans="T", lower=False).T
        R2 = scipy.linalg.cholesky(gram(Q1, Q1), lower=False)
        R = R2 @ R1
        for r_kk in np.diagonal(R):
            if np.isclose(r_kk, 0, atol=1e-8):
                print("A is rank deficient")
        z = scipy.linalg.solve_triangular(R, gram(A, y[:, None])[:, 0], trans="T", lower=False)
        return scipy.linalg.solve_triangular(R, z)
    return lls


def slab_variant(N, P):
    """(lls, update) with every reduction split into the row slabs of a P-rank run, summed in rank order."""
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import row_partition
    sl = [slice(r0 * N, (r0 + nr) * N) for r0, nr in (row_partition(N, P, p) for p in range(P))]

    def bdot(a, b):
        s = 0.0
        for q in sl:
            s = s + float(np.dot(a[q], b[q]))
        return s

    def lls(A, y):
        Rs = [scipy.linalg.qr(np.hstack([A[q], y[q][:, None]]), mode="economic")[1] for q in sl]
        R2 = scipy.linalg.qr(np.vstack(Rs), mode="r")[0]
        k = A.shape[1]
        for r_kk in np.diagonal(R2[:k, :k]):
            if np.isclose(r_kk, 0, atol=1e-8):
                print("A is rank deficient")
        return scipy.linalg.solve_triangular(R2[:k, :k], R2[:k, k])

    def update(self, jac_ev, res_ev):
        if self.basis.shape[0] == self.basis.shape[1]:
            raise O.GeneralizedKrylowSubspaceSpansEntireSpace
        g = -(jac_ev.T @ res_ev)
        h = np.array([bdot(self.basis[:, j], g) for j in range(self.basis.shape[1])])
        g = g - self.basis @ h
        if np.allclose(g, 0, atol=1e-8, rtol=0):
            raise O.GeneralizedKrylowSubspaceBreakdown("breakdown")
        g = g / np.sqrt(bdot(g, g))
        self.basis = np.hstack([self.basis, g.reshape(-1, 1)])
    return lls, update


def armijo_sums(total):
    """ref:armijo_goldstein.py:46-70 with its three sums of squares (the previous loss, each trial's loss,
    ||J d||^2) evaluated by ``total`` -- an algebraically equivalent summation (exactly rounded, or over
    row blocks in order, the device's per-block partials)."""
    def armijo(res, x, res_ev, jac_ev, args, d, max_iter=100, initial_step_length=1.0):
        t = initial_step_length
        prev = total(res_ev ** 2)
        jdd = total((jac_ev @ d) ** 2)
        for it in range(max_iter):
            cur_res = res(x + t * d, *args)
            if prev - total(cur_res ** 2) >= 0.5 * t * jdd:
                return t, cur_res, it + 1
            t /= 2
        return _ARMIJO(res, x, res_ev, jac_ev, args, d, max_iter, initial_step_length)   # raises as the reference
    return armijo


def _blocked_sum(P):
    def total(a):
        edges = np.linspace(0, a.size, P + 1).astype(int)
        s = 0.0
        for lo, hi in zip(edges[:-1], edges[1:]):
            s = s + float(np.sum(a[lo:hi]))
        return s
    return total


def variants(N, slabs=False, armijo=False):
    v = {"base": (_LLS, _UPDATE), "exact_k1": (lls_variant(True, None), _UPDATE),
         "perm7": (lls_variant(False, 7), _UPDATE), "perm8+k1": (lls_variant(True, 8), _UPDATE),
         "cholqr2": (cholqr2_lls, _UPDATE)}
    v.update({f"cholqr2b{P}": (cholqr2_blocked(P), _UPDATE) for P in (4, 64, 256)})
    if slabs:
        v.update({f"slab{P}": slab_variant(N, P) for P in range(2, 9)})
    if armijo:
        # the Armijo-Goldstein sums themselves re-rounded (round 5): a converged step's trial count is
        # decided by them, so they belong in the family that bounds it
        fsum = armijo_sums(math.fsum)
        v.update({"armijo_fsum": (_LLS, _UPDATE, fsum), "armijo_fsum+k1": (lls_variant(True, None), _UPDATE, fsum),
                  "armijo_fsum+cholqr2": (cholqr2_lls, _UPDATE, fsum)})
        v.update({f"armijo_b{P}": (_LLS, _UPDATE, armijo_sums(_blocked_sum(P))) for P in (8, 64, 512)})
        v.update({f"perm{s}": (lls_variant(False, s), _UPDATE) for s in range(9, 31)})
        v.update({f"cholqr2b{P}+armijo_fsum": (cholqr2_blocked(P), _UPDATE, fsum) for P in (64, 256)})
    return v


def trajectory(prob, y, u0, lls, update, threads, armijo=None, **kw):
    res = prob.make_res(y)
    xs, rs, nf = [], [], []
    O.linear_least_squares = lls
    if update is not _UPDATE:
        O.KrylovBasis.update = update
    if armijo is not None:
        O.armijo_goldstein = armijo
    try:
        with threadpool_limits(limits=threads, user_api="blas"), contextlib.redirect_stdout(io.StringIO()):
            O.gauss_newton_krylow(res, u0, prob.make_jac(), callback=lambda x, nfev, cg_iter: (
                xs.append(np.linalg.norm(x)), rs.append(np.linalg.norm(res(x))), nf.append(nfev)), **kw)
    except O.StepLengthConvergenceError:
        pass
    finally:
        O.linear_least_squares = _LLS
        O.armijo_goldstein = _ARMIJO
        if update is not _UPDATE:
            O.KrylovBasis.update = _UPDATE
    return np.array(xs), np.array(rs), nf


JOBS = int(os.environ.get("SENS_JOBS", "1"))      # variants run in this many forked processes


def _run_one(job):
    name, t = job
    spec = _JOBSPEC["variants"][name]
    return f"{name}@{t}", trajectory(*_JOBSPEC["inputs"], *spec[:2], t, *spec[2:], **_JOBSPEC["kw"])


_JOBSPEC = {}


ONLY = None            # --only v1,v2: recompute these variants (and base) and merge into the stored case


def envelope(N, ref=None, slabs=False, threads=THREADS, armijo=False, **kw):
    """Per-variant and maximal per-iteration distances from ``ref`` = (xnorm, rnorm) (None: the
    1-thread base oracle)."""
    prob, y, u0 = O.bratu_workload(N)
    vs = variants(N, slabs, armijo)
    jobs = [(name, t) for name in vs for t in threads
            if ONLY is None or name in ONLY or (name == "base" and ref is None)]
    _JOBSPEC.update(variants=vs, inputs=(prob, y, u0), kw=kw)
    if JOBS > 1:
        import multiprocessing as mp
        with mp.get_context("fork").Pool(JOBS) as pool:
            runs = dict(pool.map(_run_one, jobs, chunksize=1))
    else:
        runs = dict(map(_run_one, jobs))
    if ref is None:
        ref = runs[f"base@{threads[0]}"][:2]
    ref_x, ref_r = np.asarray(ref[0]), np.asarray(ref[1])
    out = {}
    for name, (xs, rs, nf) in runs.items():
        n = min(len(xs), len(ref_x))
        sx, sr = (xs[:n] - ref_x[:n]) / np.abs(ref_x[:n]), (rs[:n] - ref_r[:n]) / np.abs(ref_r[:n])
        out[name] = {"x": np.abs(sx).tolist(), "r": np.abs(sr).tolist(), "xs": sx.tolist(), "rs": sr.tolist(),
                     "nfev": nf}
    res = {"N": N, "kwargs": kw, "threads": list(threads), "variants": out}
    _summarise(res)
    return res


def _summarise(case):
    """envelope (max |distance|) and, over the variants with signed distances, diameter (spread)."""
    vs = case["variants"].values()
    n = min(len(v["x"]) for v in vs)
    case["envelope"] = {k: [max(v[k][i] for v in vs if k in v) for i in range(n)] for k in ("x", "r")}
    signed = [v for v in vs if "xs" in v]
    if signed:
        m = min(len(v["xs"]) for v in signed)
        case["diameter"] = {k: [max(0.0, max(v[k + "s"][i] for v in signed)) - min(0.0, min(v[k + "s"][i] for v in signed))
                                for i in range(m)] for k in ("x", "r")}


def _cg_with(dot):
    """O.scipy_cg with every dot product / norm by ``dot`` (an equivalent summation order)."""
    def cg(matvec, b, psolve=None, rtol=1e-5, maxiter=None, callback=None):
        norm = lambda a: math.sqrt(dot(a, a))          # noqa: E731
        bnrm2 = norm(b)
        atol = max(0.0, float(rtol) * float(bnrm2))
        if bnrm2 == 0:
            return b, 0
        maxiter = len(b) * 10 if maxiter is None else maxiter
        x, r, rho_prev, p = np.zeros_like(b), b.copy(), None, None
        for it in range(maxiter):
            if norm(r) < atol:
                return x, 0
            z = r if psolve is None else psolve(r)
            rho = dot(r, z)
            if it > 0:
                p *= rho / rho_prev
                p += z
            else:
                p = z.copy()
            q = matvec(p)
            alpha = rho / dot(p, q)
            x += alpha * p
            r -= alpha * q
            rho_prev = rho
            if callback:
                callback(x)
        return x, maxiter
    return cg


def gn_envelope(N, threads=THREADS, **kw):
    """Gauss-Newton + CGLS (ref:gauss_newton.py): the reference's CG with its dot products summed in
    other orders -- numpy pairwise, reversed, P-slab blocks in rank order (P = 2..8) -- and at 1 / 8
    BLAS threads; distances of ||x_k|| from the 1-thread reference."""
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import row_partition
    prob, y, u0 = O.bratu_workload(N)

    def slab_dot(P):
        sl = [slice(r0 * N, (r0 + nr) * N) for r0, nr in (row_partition(N, P, p) for p in range(P))]
        return lambda a, b: sum((float(np.dot(a[q], b[q])) for q in sl), 0.0)

    variants = {"base": O.scipy_cg, "pairwise": _cg_with(lambda a, b: float(np.sum(a * b))),
                "reversed": _cg_with(lambda a, b: float(np.dot(a[::-1], b[::-1])))}
    variants.update({f"slab{P}": _cg_with(slab_dot(P)) for P in range(2, 9)})
    if os.environ.get("GN_VARIANTS"):                  # (tooling: a subset, e.g. for a quick recompute)
        keep = set(os.environ["GN_VARIANTS"].split(","))
        variants = {k: v for k, v in variants.items() if k in keep or k == "base"}

    def traj(cg, t):
        xs = []
        orig = O.scipy_cg
        O.scipy_cg = cg
        try:
            with threadpool_limits(limits=t, user_api="blas"), contextlib.redirect_stdout(io.StringIO()):
                O.gauss_newton(prob.make_res(y), u0, prob.make_jac(),
                               callback=lambda x, nfev, cg_iter: xs.append(np.linalg.norm(x)), **kw)
        finally:
            O.scipy_cg = orig
        return np.array(xs)

    runs = {f"{name}@{t}": traj(cg, t) for name, cg in variants.items() for t in (threads if name == "base" else (1,))}
    ref = runs[f"base@{threads[0]}"]
    out = {}
    for name, xs in runs.items():
        n = min(len(xs), len(ref))
        sx = (xs[:n] - ref[:n]) / np.abs(ref[:n])
        out[name] = {"x": np.abs(sx).tolist(), "xs": sx.tolist(), "r": [0.0] * n, "rs": [0.0] * n}
    res = {"N": N, "kwargs": kw, "threads": list(threads), "variants": out}
    _summarise(res)
    return res


def mispredict_envelope(N):
    """tests/test_mispredict.py's injected run (a rejected first trial at iteration 12, a breakdown at
    15, ref:armijo_goldstein.py:53-62, ref:krylow.py:66-69) under the non-slab reorderings."""
    from tests.test_mispredict import injected
    prob, y, u0 = O.bratu_workload(N)
    kw = dict(krylow_restart=20, max_iter=22, version="res_old")
    runs = {}
    for name, (lls, upd) in variants(N).items():
        for t in THREADS:
            with injected():
                runs[f"{name}@{t}"] = trajectory(prob, y, u0, lls, upd, t, **kw)
    ref_x, ref_r = runs[f"base@{THREADS[0]}"][:2]
    out = {}
    for name, (xs, rs, nf) in runs.items():
        n = min(len(xs), len(ref_x))
        sx, sr = (xs[:n] - ref_x[:n]) / np.abs(ref_x[:n]), (rs[:n] - ref_r[:n]) / np.abs(ref_r[:n])
        out[name] = {"x": np.abs(sx).tolist(), "r": np.abs(sr).tolist(), "xs": sx.tolist(), "rs": sr.tolist(),
                     "nfev": nf}
    res = {"N": N, "kwargs": kw, "threads": list(THREADS), "variants": out}
    _summarise(res)
    return res


def _golden(name):
    c = json.load(open(os.path.join(OUT, "golden.json")))["cases"][name]["per_iter"]
    return c["xnorm"], c["rnorm"]


def _large(fixture, version):
    c = json.load(open(os.path.join(OUT, f"large_{fixture}.json")))["cases"][version]["per_iter"]
    return c["xnorm"], c["rnorm"]


CASES = {
    # BASELINE sizes vs the reference's own fixtures (make_golden_large.py)
    "c2_res_old": lambda: envelope(1024, _large("c2", "res_old"), armijo=True, krylow_restart=20, max_iter=100,
                                   version="res_old"),
    "c2_res_new": lambda: envelope(1024, _large("c2", "res_new"), krylow_restart=20, max_iter=100, version="res_new"),
    "head8192": lambda: envelope(8192, _large("head8192", "res_old"), threads=(4, 8), krylow_restart=20, max_iter=5,
                                 version="res_old"),
    # golden N = 100 restart-20 runs (tests/test_gpu_solvers.py)
    **{f"bratu100_r20_{v}": (lambda v=v: envelope(100, _golden(f"bratu100_{v}_r20"), slabs=True, krylow_restart=20,
                                                  max_iter=100, version=v)) for v in ("res_old", "res_new")},
    # short restart cycles at N = 256 (oracle reference)
    **{f"short256_r{r}_{v}": (lambda r=r, v=v: envelope(256, None, slabs=True, krylow_restart=r, max_iter=40, version=v))
       for r, v in ((3, "res_old"), (7, "res_old"), (5, "res_new"))},
    # multi-slab GPU test cases (tests/multislab_worker.py): single-rank oracle reference
    **{f"multislab{N}_{v}": (lambda N=N, v=v: envelope(N, None, slabs=True, krylow_restart=20, max_iter=45, version=v))
       for N in (256, 384) for v in ("res_old", "res_new", "jac_old_res_old", "jac_old_res_new")},
    # the injected misprediction run of tests/test_mispredict.py
    "mispredict1024": lambda: mispredict_envelope(1024),
    # multi-slab GN + CGLS cases (tests/multislab_worker.py)
    **{f"gn{N}": (lambda N=N: gn_envelope(N, max_iter=4, cg_rtol=1e-4)) for N in (256, 384)},
    **{f"gn{N}_pre": (lambda N=N: gn_envelope(N, max_iter=3, cg_rtol=1e-4, cg_preconditioner=True)) for N in (256, 384)},
}


def store(case, res):
    allc = json.load(open(PATH)) if os.path.exists(PATH) else {}
    if ONLY is not None and case in allc:                  # merge the recomputed variants
        old = allc[case]
        old["variants"].update(res["variants"])
        _summarise(old)
        res = old
    allc[case] = res
    with open(PATH, "w") as f:
        json.dump(allc, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--only":
        ONLY = set(args[1].split(","))
        args = args[2:]
    names = list(CASES) if args == ["all"] else args
    for case in names:
        r = CASES[case]()
        store(case, r)
        print(case, "max envelope x", max(r["envelope"]["x"]), file=sys.stderr, flush=True)
