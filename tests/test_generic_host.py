"""Generic problems through the device solver's host logic, on CPU.

``gauss_newton_krylow`` with plain NumPy ``res`` / ``jac`` callables (the reference's Rosenbrock
chain, ref:rosenbrock_problem.py:8-19, restated in oracle/) runs generic.HostCallableOps against
the NumPy test double of the C-ABI and must reproduce the reference's golden Rosenbrock runs:
stdout, exceptions and bookkeeping exact, per-iteration ||x_k|| within 1e-10 (p = 2) / 1e-9
(p = 1000, as the oracle's own pin).
"""
import contextlib
import io

import numpy as np
import pytest

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
from oracle import gnk_oracle as O
from tests.numpy_backend import NumpyBackend
from tests.test_oracle_golden import _check, _run


def rosen_x0(arr, p, name):
    if p == 2:
        return np.array({"m1_1": [-1.0, 1.0], "2_2": [2.0, 2.0]}[name])
    x = {"i": arr["rosen1000_x0_i"], "ii": 2 * np.ones(1000), "iii": 2 * np.ones(1000)}[name].copy()
    if name == "iii":
        x[2] = 1.99
    return x


@pytest.mark.parametrize("p,x0name", [(2, "m1_1"), (2, "2_2"), (1000, "i"), (1000, "ii"), (1000, "iii")])
@pytest.mark.parametrize("version", ["res_old", "res_new", "gn"])
def test_generic_gnk_rosenbrock(golden, p, x0name, version):
    meta, arr = golden
    res, jac = O.rosenbrock(p)
    x0 = rosen_x0(arr, p, x0name)
    x0_copy = x0.copy()
    if version == "gn":
        out, rec, so, exc = _run(gnk.gauss_newton, res, x0, jac, _backend=NumpyBackend())
    else:
        out, rec, so, exc = _run(gnk.gauss_newton_krylow, res, x0, jac, version=version, _backend=NumpyBackend())
    name = f"rosen{p}_{x0name}_{version}"
    _check(meta["cases"][name], out, rec, so, exc, rtol=1e-10 if p == 2 else 1e-9)
    np.testing.assert_array_equal(x0, x0_copy)        # x0 is not mutated
    if p == 2:
        np.testing.assert_allclose(out.x, arr[name + "__x"], rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("p,x0", [(2, [2.0, 2.0]), (2, [-1.0, 1.0]), (10, None), (40, None)])
def test_generic_gn_dense_jacobian_lstsq_branch(p, x0):
    """gauss_newton with an ndarray Jacobian (ref:gauss_newton.py:115-116): the device
    CholeskyQR solve vs scipy.linalg.lstsq in the oracle (the reference's own call) -- bookkeeping
    and cg_iter (None) exact, ||x_k|| within 1e-10, no rank messages."""
    res, jac = O.rosenbrock(p)
    djac = lambda x: jac(x).toarray()  # noqa: E731
    x0 = np.asarray(x0) if x0 is not None else np.random.default_rng(p).uniform(-1.5, 1.5, p)
    ra, rb = [], []
    out_a = io.StringIO()
    with contextlib.redirect_stdout(out_a):
        a = gnk.gauss_newton(res, x0, djac, _backend=NumpyBackend(),
                             callback=lambda x, nfev, cg_iter: ra.append((np.linalg.norm(x), nfev, cg_iter)))
    out_b = io.StringIO()
    with contextlib.redirect_stdout(out_b):
        b = O.gauss_newton(res, x0, djac,
                           callback=lambda x, nfev, cg_iter: rb.append((np.linalg.norm(x), nfev, cg_iter)))
    assert out_a.getvalue() == out_b.getvalue()
    assert (a.nit, a.nrev, a.njev, a.success) == (b.nit, b.nrev, b.njev, b.success)
    assert [r[1:] for r in ra] == [r[1:] for r in rb]
    np.testing.assert_allclose([r[0] for r in ra], [r[0] for r in rb], rtol=1e-10)
    np.testing.assert_allclose(a.x, b.x, rtol=1e-9, atol=1e-12)


def test_generic_args_and_dense_jacobian():
    """res(x, *args) / jac(x, *args) with an ndarray Jacobian (the reference accepts both)."""
    res, jac = O.rosenbrock(2)
    out = gnk.gauss_newton_krylow(lambda x, s: s * res(x), np.array([2.0, 2.0]),
                                  lambda x, s: s * jac(x).toarray(), args=(1.0,), _backend=NumpyBackend())
    ref = O.gauss_newton_krylow(res, np.array([2.0, 2.0]), jac)
    assert (out.nit, out.nrev, out.njev, out.success) == (ref.nit, ref.nrev, ref.njev, ref.success)
    np.testing.assert_allclose(out.x, ref.x, rtol=1e-12)


# -- rank-deficient Jacobians (the lstsq branch must not fail when no Cholesky factor exists)
def _rank1_problem():
    """3 residuals, 2 parameters, J = a(s) b^T of rank 1 everywhere (s = x0 + 2 x1), nonzero residual."""
    def res(x):
        s = x[0] + 2 * x[1]
        return np.array([np.exp(s) - 2.0, s * s - 0.3, 0.5 * s - 0.2])

    def jac(x):
        s = x[0] + 2 * x[1]
        return np.outer([np.exp(s), 2 * s, 0.5], [1.0, 2.0])
    return res, jac


def _trace(fn, res, x0, jac, **kw):
    rec, so = [], io.StringIO()
    exc = None
    try:
        with contextlib.redirect_stdout(so):
            out = fn(res, x0, jac, callback=lambda x, nfev, cg_iter: rec.append((x.copy(), nfev, cg_iter)), **kw)
    except Exception as e:            # noqa: BLE001 -- the reference's exception types are compared
        out, exc = None, e
    return out, rec, so.getvalue(), exc


def check_rank_deficient_gn(backend_kw):
    """gauss_newton's lstsq branch (ref:gauss_newton.py:115-116) on a rank-1 Jacobian: scipy.linalg.lstsq
    returns the minimum-norm step; the device CholeskyQR solve takes R's truncated-SVD solution with
    lstsq's cut-off (lls.CholQR2Solver, min_norm_if_singular).  Bookkeeping exact, iterates 1e-10."""
    res, jac = _rank1_problem()
    a = _trace(gnk.gauss_newton, res, np.array([0.1, 0.1]), jac, **backend_kw)
    b = _trace(O.gauss_newton, res, np.array([0.1, 0.1]), jac)
    assert a[3] is None and b[3] is None
    assert (a[0].nit, a[0].nrev, a[0].njev, a[0].success) == (b[0].nit, b[0].nrev, b[0].njev, b[0].success)
    assert [r[1:] for r in a[1]] == [r[1:] for r in b[1]]
    np.testing.assert_allclose(np.array([r[0] for r in a[1]]), np.array([r[0] for r in b[1]]), rtol=1e-10, atol=1e-14)
    assert a[2] == b[2]
    # a linear rank-1 least-squares problem (the advisor's case): the first step is lstsq's minimum-norm
    # solution; the second step's direction is rounding noise (reference: ||d|| = 6e-17 and 100 failed
    # halvings), so only the step and the end state are compared -- either outcome of that tie
    A = np.array([[1.0, 2.0], [2.0, 4.0], [3.0, 6.0]])
    y = np.array([1.0, 0.0, 2.0])
    a = _trace(gnk.gauss_newton, lambda x: y - A @ x, np.array([1.0, 1.0]), lambda x: -A, **backend_kw)
    b = _trace(O.gauss_newton, lambda x: y - A @ x, np.array([1.0, 1.0]), lambda x: -A)
    np.testing.assert_allclose(a[1][0][0], b[1][0][0], rtol=0, atol=1e-14)
    assert a[1][0][1] == b[1][0][1]
    assert a[3] is None or type(a[3]).__name__ == type(b[3]).__name__ == "StepLengthConvergenceError"
    np.testing.assert_allclose(a[1][-1][0], b[1][0][0], rtol=0, atol=1e-14)


def check_rank_deficient_gnk(backend_kw):
    """gauss_newton_krylow on a rank-1 Jacobian: the first step (k = 1) matches; at k = 2, J V has rank 1 and
    the reference's QR prints 'A is rank deficient' (ref:gauss_newton_krylow.py:32-34) before its
    rounding-noise step -- the message and the SpansEntireSpace warning must come out the same way."""
    res, jac = _rank1_problem()
    a = _trace(gnk.gauss_newton_krylow, res, np.array([0.1, 0.1]), jac, **backend_kw)
    b = _trace(O.gauss_newton_krylow, res, np.array([0.1, 0.1]), jac)
    np.testing.assert_allclose(a[1][0][0], b[1][0][0], rtol=1e-12)
    assert a[1][0][1] == b[1][0][1]
    head = ("A is rank deficient\nWarning: The genearlized krylow subspace is now identical to the whole "
            "parameter space at iteration = 2\n")
    assert a[2].startswith(head) and b[2].startswith(head)


def test_rank_deficient_dense_gn():
    check_rank_deficient_gn(dict(_backend=NumpyBackend()))


def test_rank_deficient_gnk():
    check_rank_deficient_gnk(dict(_backend=NumpyBackend()))


# -- bases wider than 63 columns (the reference never restarts by default and grows the basis to
# max_iter - 1 columns, ref:gauss_newton_krylow.py:81-82, ref:krylow.py:72-73) and dense Jacobians with more
# than 63 parameters (ref:gauss_newton.py:115-116)
def check_wide_basis(backend_kw):
    """Rosenbrock p = 1000 from the F5 start, res_old, tol 1e-12, max_iter 71: 70 iterations without restart,
    the basis grows to 70 columns -- bookkeeping exact, ||x_k|| within 1e-10 of the oracle.  (At tol 0 / longer
    runs the converged steps are Armijo rounding ties; this window stops before them.)"""
    meta_arr = dict(np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "golden.npz")))
    res, jac = O.rosenbrock(1000)
    x0 = meta_arr["rosen1000_x0_i"]
    runs = []
    for fn, kw in ((gnk.gauss_newton_krylow, backend_kw), (O.gauss_newton_krylow, {})):
        rec = []
        with contextlib.redirect_stdout(io.StringIO()):
            r = fn(res, x0.copy(), jac, tol=1e-12, max_iter=71, version="res_old",
                   callback=lambda x, nfev, cg_iter: rec.append((np.linalg.norm(x), nfev)), **kw)
        runs.append((r, rec))
    (a, ra), (b, rb) = runs
    assert (a.nit, a.nrev, a.njev, a.success) == (b.nit, b.nrev, b.njev, b.success) == (70, 71, 71, False)
    assert [n for _, n in ra] == [n for _, n in rb]
    np.testing.assert_allclose([x for x, _ in ra], [x for x, _ in rb], rtol=1e-10)


def check_dense_100(backend_kw):
    """gauss_newton's lstsq branch with 100 parameters (ndarray Jacobians of the Rosenbrock chain, three
    starts) vs scipy.linalg.lstsq in the oracle: bookkeeping exact, ||x_k|| within 1e-10."""
    res, jac = O.rosenbrock(100)
    djac = lambda x: jac(x).toarray()  # noqa: E731
    rng = np.random.default_rng(42)
    for x0 in (2 * np.ones(100), 1 + 0.1 * rng.standard_normal(100), np.r_[2.0, 2.0, 1.99, 2 * np.ones(97)]):
        runs = []
        for fn, kw in ((gnk.gauss_newton, backend_kw), (O.gauss_newton, {})):
            rec = []
            with contextlib.redirect_stdout(io.StringIO()):
                r = fn(res, x0.copy(), djac, callback=lambda x, nfev, cg_iter: rec.append((np.linalg.norm(x), nfev)), **kw)
            runs.append((r, rec))
        (a, ra), (b, rb) = runs
        assert (a.nit, a.nrev, a.njev, a.success) == (b.nit, b.nrev, b.njev, b.success)
        assert [n for _, n in ra] == [n for _, n in rb]
        np.testing.assert_allclose([x for x, _ in ra], [x for x, _ in rb], rtol=1e-10)


def test_wide_basis_beyond_63_columns():
    check_wide_basis(dict(_backend=NumpyBackend()))


def test_dense_lstsq_100_parameters():
    check_dense_100(dict(_backend=NumpyBackend()))


def _graded_step(svals, backend_kw, seed=7, m=14):
    """One GN step on the linear problem y - A x, A = U diag(svals) W^T; (step, svd of A, U^T y)."""
    rng = np.random.default_rng(seed)
    p = len(svals)
    U, _ = np.linalg.qr(rng.standard_normal((m, m)))
    W, _ = np.linalg.qr(rng.standard_normal((p, p)))
    A = U[:, :p] @ np.diag(svals) @ W.T
    y = rng.standard_normal(m)
    rec = []
    with contextlib.redirect_stdout(io.StringIO()):
        try:
            gnk.gauss_newton(lambda x: y - A @ x, np.zeros(p), lambda x: -A, max_iter=2,
                             callback=lambda x, nfev, cg_iter: rec.append(x.copy()), **backend_kw)
        except Exception as e:                      # noqa: BLE001 -- the step is what is checked
            assert type(e).__name__ == "StepLengthConvergenceError", e
    assert rec, "no step taken"
    Us, ss, Vt = np.linalg.svd(A)
    return rec[0], A, y, ss, Vt, Us[:, :p].T @ y     # linear problem: the full step (t = 1) is accepted


def check_graded_spectrum_gn(backend_kw):
    """dense Jacobians with singular values far below sqrt(eps) sigma_max.  scipy.linalg.lstsq
    (gelsd, cond = eps) resolves every direction above eps sigma_max; the CholeskyQR solve only sees the
    Gram, whose shifted factors regularise the directions below ~sqrt(n k eps) sigma_max (documented in
    lls.CholQR2Solver).  What the step holds to (SVD of the computed A):
      * one such direction (1, 1e-2, 1e-4, 1e-9): the components along the resolved directions equal the
        least-squares solution's to 1e-6 (measured 1.5e-7);
      * a graded tail (1 .. 1e-14, four directions below 1e-8): the step's residual is within 1e-4 of the
        least-squares optimum (measured 4.5e-5; gelsd's own step, with 1e14-sized coefficients, lands
        1.6e-4 above it) -- but its components along the resolved directions
        deviate by up to ~5e-3 (relative) from gelsd's: the band where this branch and gelsd differ."""
    d, A, y, ss, Vt, uy = _graded_step([1.0, 1e-2, 1e-4, 1e-9], backend_kw)
    big = ss >= 1e-6 * ss[0]
    np.testing.assert_allclose(Vt[big] @ d, uy[big] / ss[big], rtol=1e-6)
    d, A, y, ss, Vt, uy = _graded_step([1.0, 1e-2, 1e-4, 1e-9, 1e-11, 1e-13, 1e-14], backend_kw)
    r_opt2 = float(y @ y - uy @ uy)                                     # min ||y - A x||^2 (SVD)
    r_dev2 = float(np.sum((y - A @ d) ** 2))
    r_ref2 = float(np.sum((y - A @ np.linalg.lstsq(A, y, rcond=None)[0]) ** 2))   # gelsd's step: 1.6e-4 above
    assert r_opt2 * (1 - 1e-10) <= r_dev2 <= r_opt2 * (1 + 1e-4), (r_dev2, r_opt2)
    assert r_dev2 <= r_ref2, (r_dev2, r_ref2)


def test_graded_spectrum_dense_gn():
    check_graded_spectrum_gn(dict(_backend=NumpyBackend()))


def test_shared_backend_across_pair_and_plain_solvers():
    """one backend serves a Bratu GN (compensated reductions as (s, c) pairs) and generic
    solvers (plain reductions) in any order -- the mode is set per call and checked against each
    output buffer's size, so neither run writes past a buffer or reads the other's layout."""
    be = NumpyBackend()
    res, jac = O.rosenbrock(1000)
    x0 = 2 * np.ones(1000)
    prob, y, u0 = O.bratu_workload(24)

    def bratu_gn(backend):
        p = gnk.BratuPdeProblem(25, 5, 10)
        with contextlib.redirect_stdout(io.StringIO()):
            return gnk.gauss_newton(p.make_res(y), u0, p.make_jac(), max_iter=4, _backend=backend)

    def generic(backend, method, **kw):
        with contextlib.redirect_stdout(io.StringIO()):
            return method(res, x0, jac, max_iter=6, _backend=backend, **kw)

    ref_gn = bratu_gn(NumpyBackend())
    ref_gen = generic(NumpyBackend(), gnk.gauss_newton)
    ref_gnk = generic(NumpyBackend(), gnk.gauss_newton_krylow, version="res_old")
    a = bratu_gn(be)
    assert be.pairs                                       # the Bratu GN left the context in pair mode
    b = generic(be, gnk.gauss_newton)
    c = generic(be, gnk.gauss_newton_krylow, version="res_old")
    d = bratu_gn(be)
    for got, ref in ((a, ref_gn), (b, ref_gen), (c, ref_gnk), (d, ref_gn)):
        assert (got.nit, got.nrev, got.njev) == (ref.nit, ref.nrev, ref.njev)
        np.testing.assert_array_equal(got.x, ref.x)


def test_reduction_buffer_checked_against_mode():
    import torch
    be = NumpyBackend()
    x = torch.ones(8, dtype=torch.float64)
    with pytest.raises(ValueError):
        be.flat_stats(x, torch.zeros(2, dtype=torch.float64), pairs=True)     # pair mode writes 3
    with pytest.raises(ValueError):
        be.flat_dot(x, x, torch.zeros(1, dtype=torch.float64), pairs=True)   # pair mode writes 2
