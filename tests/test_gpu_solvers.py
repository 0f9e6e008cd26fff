"""End-to-end parity of the device solvers (HIP path) with the reference's golden runs.

Bookkeeping (nit / njev / success / per-iteration nfev / printed messages) exact;
per-iteration ||x_k|| within 1e-10 relative, ||r_k|| within 1e-10 of ||r_0||.
Known-fragile: the restart-20 runs' final converged step, whose
Armijo test is a rounding tie -- only that step's trial count may differ.
"""
import contextlib
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from oracle import gnk_oracle as O  # noqa: E402
from tests import tolerances as T  # noqa: E402
from tests.test_host_logic import check  # noqa: E402


def run(method, prob_kw, u0, y, **kw):
    prob = gnk.BratuPdeProblem(**prob_kw)
    ref_res = O.BratuPdeProblem(**prob_kw).make_res(y)
    rec = {"xnorm": [], "rnorm": [], "nfev": [], "cg_iter": []}

    def cb(x, nfev, cg_iter):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(ref_res(x))))
        rec["nfev"].append(nfev)
        rec["cg_iter"].append(cg_iter)

    buf = io.StringIO()
    exc = None
    out = None
    with contextlib.redirect_stdout(buf):
        try:
            out = method(prob.make_res(y), u0, prob.make_jac(), callback=cb, **kw)
        except gnk.StepLengthConvergenceError as e:
            exc = ["StepLengthConvergenceError", e.message]
    return out, rec, buf.getvalue().splitlines(), exc


@pytest.mark.parametrize("version", ["res_old", "res_new", "jac_old_res_old", "jac_old_res_new"])
@pytest.mark.parametrize("restart", [None, 20])
def test_gnk_bratu24(golden, version, restart):
    meta, arr = golden
    out, rec, so, exc = run(gnk.gauss_newton_krylow, dict(grid_nodes=25, ALPHA=5, LAMBDA=10),
                            arr["bratu24_u0"], arr["bratu24_y"], version=version, max_iter=100,
                            krylow_restart=restart)
    check(meta["cases"][f"bratu24_{version}_r{restart}"], out, rec, so, exc, fragile_last=restart is not None)
    if restart is None:
        np.testing.assert_allclose(out.x, arr[f"bratu24_{version}_rNone__x"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("version", ["res_old", "res_new"])
@pytest.mark.parametrize("restart", [None, 20])
def test_gnk_bratu100(golden, version, restart):
    meta, arr = golden
    prob = O.BratuPdeProblem(101, 5, 10)
    y = prob.pde_operator(prob.u_true)
    out, rec, so, exc = run(gnk.gauss_newton_krylow, dict(grid_nodes=101, ALPHA=5, LAMBDA=10),
                            arr["bratu100_u0"], y, version=version, max_iter=100, krylow_restart=restart)
    case = meta["cases"][f"bratu100_{version}_r{restart}"]
    if restart is None:
        check(case, out, rec, so, exc, rtol=T.NORTH_STAR)
        np.testing.assert_allclose(out.x, arr[f"bratu100_{version}_r{restart}__x"], rtol=0,
                                   atol=1e-9 * np.abs(out.x).max())
        return
    # restart 20: per-iteration bound max(1e-10, what reordering the reference's own QR / sums moves
    # it by) -- tests/tolerances.py, case bratu100_r20_<version>
    tol = T.per_iteration(f"bratu100_r20_{version}", len(case["per_iter"]["xnorm"]))
    check(case, out, dict(rec, xnorm=case["per_iter"]["xnorm"], rnorm=case["per_iter"]["rnorm"]), so, exc)
    ex = np.abs(np.array(rec["xnorm"]) - case["per_iter"]["xnorm"]) / np.abs(case["per_iter"]["xnorm"])
    assert np.all(ex <= tol), (ex.max(), np.nonzero(ex > tol))
    tol_r = T.per_iteration(f"bratu100_r20_{version}", len(case["per_iter"]["rnorm"]), "r")
    er = np.abs(np.array(rec["rnorm"]) - case["per_iter"]["rnorm"]) / np.abs(case["per_iter"]["rnorm"])
    assert np.all(er <= tol_r), (er.max(), np.nonzero(er > tol_r))
    np.testing.assert_allclose(out.x, arr[f"bratu100_{version}_r{restart}__x"], rtol=0,
                               atol=10 * tol[-1] * np.abs(out.x).max())


@pytest.mark.parametrize("version", ["res_old", "res_new"])
def test_gnk_noscale(golden, version):
    meta, _ = golden
    prob, y, u0 = O.bratu_workload(24, grid_resolution=1)
    out, rec, so, exc = run(gnk.gauss_newton_krylow, dict(grid_nodes=25, ALPHA=5, LAMBDA=10, grid_resolution=1),
                            u0, y, version=version, max_iter=100)
    check(meta["cases"][f"bratu24_noscale_{version}"], out, rec, so, exc)


def test_gnk_linear_breakdown(golden):
    meta, arr = golden
    prob = O.BratuPdeProblem(25, 5, 0.0)
    y = prob.pde_operator(prob.u_true)
    out, rec, so, exc = run(gnk.gauss_newton_krylow, dict(grid_nodes=25, ALPHA=5, LAMBDA=0.0),
                            arr["bratu24_linear_u0"], y, max_iter=100)
    case = meta["cases"]["bratu24_linear_res_old"]
    assert so == case["stdout"]                     # breakdown at iteration 2, basis (576, 2)
    # Iteration 3 re-solves the least-squares problem of iteration 2 (linear problem, same basis):
    # d is rounding noise (reference: ||d|| = 3e-17) and the Armijo outcome is a rounding tie
    # ("assert only the breakdown event").  The reference sees c + t d == c for
    # every t and fails 100 halvings; a noise step that survives the addition is accepted and
    # then meets the convergence test at once.  Either way the iterate is the reference's.
    if exc is not None:
        assert exc[0] == "StepLengthConvergenceError"
    else:
        assert out.success and out.nit == 3
        assert rec["nfev"][:2] == case["per_iter"]["nfev"]
        np.testing.assert_allclose(rec["xnorm"][2], case["per_iter"]["xnorm"][1], rtol=1e-12)
    np.testing.assert_allclose(rec["xnorm"][:2], case["per_iter"]["xnorm"], rtol=1e-10)


def test_gnk_linear_res_new(golden):
    """Chaotic near-breakdown trajectory (tests/test_oracle_sensitivity.py): a 1e-13 relative
    perturbation of the reference's own step moves ||x_k|| by ~1e-4 around iteration 87.
    Bookkeeping exact; ||x_k|| at 1e-10 before the sensitive phase (k < 30) and at the end;
    inside it, within the reference's own perturbation envelope (1e-3)."""
    meta, arr = golden
    prob = O.BratuPdeProblem(25, 5, 0.0)
    y = prob.pde_operator(prob.u_true)
    out, rec, so, exc = run(gnk.gauss_newton_krylow, dict(grid_nodes=25, ALPHA=5, LAMBDA=0.0),
                            arr["bratu24_linear_u0"], y, version="res_new", max_iter=200)
    case = meta["cases"]["bratu24_linear_res_new"]
    assert so == case["stdout"] and exc is None
    assert (out.nit, out.nrev, out.njev, out.success) == (case["nit"], case["nrev"], case["njev"], case["success"])
    ref = case["per_iter"]
    assert rec["nfev"] == ref["nfev"]
    x, xr = np.array(rec["xnorm"]), np.array(ref["xnorm"])
    np.testing.assert_allclose(x[:30], xr[:30], rtol=1e-10)
    np.testing.assert_allclose(x, xr, rtol=1e-3)
    np.testing.assert_allclose(x[-3:], xr[-3:], rtol=1e-10)


@pytest.mark.parametrize("name,kw", [("bratu24_gn", {}), ("bratu24_gn_precond", {"cg_preconditioner": True})])
def test_gn_bratu24(golden, name, kw):
    meta, arr = golden
    out, rec, so, exc = run(gnk.gauss_newton, dict(grid_nodes=25, ALPHA=5, LAMBDA=10),
                            arr["bratu24_u0"], arr["bratu24_y"], **kw)
    check(meta["cases"][name], out, rec, so, exc, rtol=1e-9)


def test_gn_bratu100(golden):
    """CG runs of 900-2000 iterations (unpreconditioned + Jacobi, ref:gauss_newton.py:45-58): the device
    dot products are compensated (exactly rounded sums), which reproduces the reference's cg_iter of
    every outer step; bookkeeping exact, iterates within 1e-10."""
    meta, arr = golden
    prob = O.BratuPdeProblem(101, 5, 10)
    y = prob.pde_operator(prob.u_true)
    out, rec, so, exc = run(gnk.gauss_newton, dict(grid_nodes=101, ALPHA=5, LAMBDA=10), arr["bratu100_u0"], y)
    case = meta["cases"]["bratu100_gn"]
    check(case, out, dict(rec, rnorm=case["per_iter"]["rnorm"]), so, exc, rtol=T.NORTH_STAR)
    # ||r_k|| = ||y - F(x_k)|| is a difference of vectors of norm ~||y||: near convergence (||r|| ~ 1e-7 of
    # ||y||) its relative value amplifies the iterates' 1e-10 by ||J|| ||x|| / ||r||, so it is held to
    # 1e-10 of ||y|| (absolute), the accuracy any evaluation of the residual has
    np.testing.assert_allclose(rec["rnorm"], case["per_iter"]["rnorm"], rtol=0, atol=T.NORTH_STAR * np.linalg.norm(y))


@pytest.mark.parametrize("N,name", [(24, "bratu24_gn"), (100, "bratu100_gn")])
def test_gn_single_reduction_cg_gpu(golden, N, name):
    """cg_variant="single_reduction" (Chronopoulos-Gear: one reduction per CG iteration) --
    a NON-parity option: a different recurrence from the reference's scipy cg (same iterates only in
    exact arithmetic), so a long solve may stop one iteration apart and the iterates differ by the
    recurrences' rounding; outer bookkeeping exact, cg_iter within 1, iterates within 1e-6."""
    meta, arr = golden
    if N == 24:
        u0, y = arr["bratu24_u0"], arr["bratu24_y"]
    else:
        u0, y = arr["bratu100_u0"], O.BratuPdeProblem(101, 5, 10).pde_operator(O.BratuPdeProblem(101, 5, 10).u_true)
    out, rec, so, exc = run(gnk.gauss_newton, dict(grid_nodes=N + 1, ALPHA=5, LAMBDA=10), u0, y,
                            cg_variant="single_reduction")
    case = meta["cases"][name]
    assert so == case["stdout"] and exc is None
    assert (out.nit, out.nrev, out.njev, out.success) == (case["nit"], case["nrev"], case["njev"], case["success"])
    ref = case["per_iter"]
    assert rec["nfev"] == ref["nfev"]
    assert all(abs(a - b) <= 1 for a, b in zip(rec["cg_iter"], ref["cg_iter"]))
    np.testing.assert_allclose(rec["xnorm"], ref["xnorm"], rtol=1e-6)


@pytest.mark.parametrize("N", [24, 100])
@pytest.mark.parametrize("pre,rtol", [(False, 1e-4), (True, 1e-4), (True, 1e-8)])
def test_cg_least_squares(golden, N, pre, rtol):
    meta, arr = golden
    prob, y, u0 = O.bratu_workload(N)
    r0 = prob.make_res(y)(u0)
    dprob = gnk.BratuPdeProblem(N + 1, 5, 10)
    x, it = gnk.cg_least_squares(-1 * dprob.make_jac()(u0), r0, cg_rtol=rtol, preconditioner=pre)
    name = f"cgls{N}_pre{int(pre)}" + ("_rtol1e-8" if rtol == 1e-8 else "")
    assert it == meta["cases"][name]["cg_iter"]
    # compensated device dot products: the short solves agree to 1e-10 of max |x|; the 949-iteration
    # rtol 1e-8 solve to CGLS_LONG_X, which the exactly rounded recurrence itself is from the
    # reference's (tests/tolerances.py)
    tol = T.CGLS_LONG_X if it > 500 else T.NORTH_STAR
    np.testing.assert_allclose(x, arr[name + "__x"], rtol=0, atol=tol * np.abs(x).max())


def test_drop_in_closures_on_host_arrays(golden):
    """make_res / make_jac results still behave like the reference closures on NumPy arrays."""
    meta, arr = golden
    prob = gnk.BratuPdeProblem(65, 5, 10)
    u, v, w = arr["ops64_u"], arr["ops64_v"], arr["ops64_w"]
    J = prob.make_jac()(u)
    np.testing.assert_allclose(J @ v, arr["ops64_Jv"], rtol=1e-13, atol=1e-13 * np.abs(arr["ops64_Jv"]).max())
    np.testing.assert_allclose(J.T @ w, arr["ops64_JTw"], rtol=1e-13, atol=1e-13 * np.abs(arr["ops64_JTw"]).max())
    np.testing.assert_allclose(prob.pde_operator(u), arr["ops64_F"], rtol=1e-13,
                               atol=1e-13 * np.abs(arr["ops64_F"]).max())
    np.testing.assert_allclose(prob.make_res(arr["ops64_y"])(u), arr["ops64_res"], rtol=1e-12,
                               atol=1e-12 * np.abs(arr["ops64_res"]).max())


def test_gnk_deterministic_restart_large():
    """N = 1024, restart 20: two runs are bitwise identical (fixed-order reductions, no atomics).  The
    trajectory itself is checked against the reference's C2 run in test_gpu_baseline_sizes.py."""
    N = 1024
    prob_o, y, u0 = O.bratu_workload(N)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    outs = []
    for _ in range(2):
        with contextlib.redirect_stdout(io.StringIO()):
            outs.append(gnk.gauss_newton_krylow(prob.make_res(y), u0, prob.make_jac(), krylow_restart=20, max_iter=25))
    np.testing.assert_array_equal(outs[0].x, outs[1].x)
    assert outs[0].nrev == outs[1].nrev


@pytest.mark.parametrize("restart,version", [(3, "res_old"), (7, "res_old"), (5, "res_new")])
def test_gnk_short_restart_cycles_vs_oracle(restart, version):
    """Short restart cycles at N = 256 exercise the speculative next-step solve across
    many restarts and loop ends: bookkeeping equal to the oracle, ||x_k|| within max(1e-10, the
    reordering envelope of the same run, tests/tolerances.py case short256_r<restart>_<version>)."""
    N = 256
    prob_o, y, u0 = O.bratu_workload(N)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    rec_d, rec_o = [], []
    with contextlib.redirect_stdout(io.StringIO()):
        out = gnk.gauss_newton_krylow(prob.make_res(y), u0, prob.make_jac(), krylow_restart=restart, max_iter=40,
                                      version=version,
                                      callback=lambda x, nfev, cg_iter: rec_d.append((np.linalg.norm(x), nfev)))
        ref = O.gauss_newton_krylow(prob_o.make_res(y), u0, prob_o.make_jac(), krylow_restart=restart, max_iter=40,
                                    version=version,
                                    callback=lambda x, nfev, cg_iter: rec_o.append((np.linalg.norm(x), nfev)))
    assert (out.nit, out.nrev, out.njev, out.success) == (ref.nit, ref.nrev, ref.njev, ref.success)
    assert [n for _, n in rec_d] == [n for _, n in rec_o]
    xd, xo = np.array([a for a, _ in rec_d]), np.array([a for a, _ in rec_o])
    tol = T.per_iteration(f"short256_r{restart}_{version}", len(xo))
    ex = np.abs(xd - xo) / np.abs(xo)
    assert np.all(ex <= tol), (ex.max(), np.nonzero(ex > tol))
