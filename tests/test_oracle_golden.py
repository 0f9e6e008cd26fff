"""Pin the CPU oracle (oracle/gnk_oracle.py) against the reference's own outputs.

The golden vectors were produced by running the reference (tests/golden/make_golden.py).
Bookkeeping (nit / nrev / njev / success / stdout) must match exactly; fp64 norms
within 1e-10 relative (the north-star tolerance), per iteration.
"""
import contextlib
import io

import numpy as np
import pytest
import scipy.sparse

from oracle import gnk_oracle as O

RTOL = 1e-10


_rosen = O.rosenbrock


def _run(method, res, x0, jac, **kw):
    rec = {"xnorm": [], "rnorm": [], "nfev": [], "cg_iter": []}

    def cb(x, nfev, cg_iter):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(res(x))))
        rec["nfev"].append(nfev)
        rec["cg_iter"].append(cg_iter)

    buf = io.StringIO()
    exc = None
    out = None
    with contextlib.redirect_stdout(buf):
        try:
            out = method(res, x0, jac, callback=cb, **kw)
        except O.StepLengthConvergenceError as e:
            exc = ["StepLengthConvergenceError", e.message]
    return out, rec, buf.getvalue().splitlines(), exc


def _check(case, out, rec, stdout, exc, norm_iters=None, rtol=RTOL):
    assert stdout == case["stdout"]
    assert exc == case["exception"]
    if out is not None:
        assert (out.nit, out.nrev, out.njev, out.success) == (case["nit"], case["nrev"], case["njev"], case["success"])
    ref = case["per_iter"]
    assert rec["nfev"] == ref["nfev"]
    assert rec["cg_iter"] == ref["cg_iter"]
    n = len(ref["xnorm"]) if norm_iters is None else min(norm_iters, len(ref["xnorm"]))
    np.testing.assert_allclose(rec["xnorm"][:n], ref["xnorm"][:n], rtol=rtol)
    # residual norms near convergence are cancellation-limited (||y - F(x)|| with
    # ||F(x)|| >> ||r||): relative to the iteration-0 residual norm
    np.testing.assert_allclose(rec["rnorm"][:n], ref["rnorm"][:n], rtol=rtol,
                               atol=RTOL * (ref["rnorm"][0] if ref["rnorm"] else 0.0))


@pytest.mark.parametrize("x0name,x0", [("m1_1", [-1.0, 1.0]), ("2_2", [2.0, 2.0])])
@pytest.mark.parametrize("version", ["res_old", "res_new", "gn"])
def test_rosenbrock_p2(golden, x0name, x0, version):
    meta, arr = golden
    res, jac = _rosen(2)
    if version == "gn":
        out, rec, so, exc = _run(O.gauss_newton, res, np.array(x0), jac)
    else:
        out, rec, so, exc = _run(O.gauss_newton_krylow, res, np.array(x0), jac, version=version)
    name = f"rosen2_{x0name}_{version}"
    _check(meta["cases"][name], out, rec, so, exc)
    np.testing.assert_allclose(out.x, arr[name + "__x"], rtol=RTOL, atol=1e-14)


@pytest.mark.parametrize("x0name", ["i", "ii", "iii"])
@pytest.mark.parametrize("version", ["res_old", "res_new", "gn"])
def test_rosenbrock_p1000(golden, x0name, version):
    meta, arr = golden
    res, jac = _rosen(1000)
    x_exact = np.ones(1000)
    x0 = {"i": arr["rosen1000_x0_i"], "ii": 2 * x_exact, "iii": 2 * x_exact}[x0name].copy()
    if x0name == "iii":
        x0[2] = 1.99
    if version == "gn":
        out, rec, so, exc = _run(O.gauss_newton, res, x0, jac)
    else:
        out, rec, so, exc = _run(O.gauss_newton_krylow, res, x0, jac, version=version)
    _check(meta["cases"][f"rosen1000_{x0name}_{version}"], out, rec, so, exc, rtol=1e-9)


@pytest.mark.parametrize("version", ["res_old", "res_new", "jac_old_res_old", "jac_old_res_new"])
@pytest.mark.parametrize("restart", [None, 20])
def test_bratu24_gnk(golden, version, restart):
    meta, arr = golden
    prob, y, u0 = O.bratu_workload(24)
    np.testing.assert_array_equal(u0, arr["bratu24_u0"])
    np.testing.assert_allclose(y, arr["bratu24_y"], rtol=1e-14, atol=1e-12)
    res, jac = prob.make_res(y), prob.make_jac()
    out, rec, so, exc = _run(O.gauss_newton_krylow, res, u0, jac, version=version,
                             krylow_restart=restart, max_iter=100)
    case = meta["cases"][f"bratu24_{version}_r{restart}"]
    # the converged res_new residual (~7e-7) is cancellation-limited: SURVEY §8c
    _check(case, out, rec, so, exc, rtol=1e-8 if restart else RTOL)


@pytest.mark.parametrize("version", ["res_old", "res_new"])
def test_bratu24_noscale(golden, version):
    meta, _ = golden
    prob, y, u0 = O.bratu_workload(24, grid_resolution=1)
    out, rec, so, exc = _run(O.gauss_newton_krylow, prob.make_res(y), u0, prob.make_jac(),
                             version=version, max_iter=100)
    _check(meta["cases"][f"bratu24_noscale_{version}"], out, rec, so, exc)


def test_bratu24_linear_breakdown(golden):
    """F4: breakdown at iteration 2 then StepLengthConvergenceError (fragile: assert events)."""
    meta, arr = golden
    prob, y, u0 = O.bratu_workload(24, lam=0.0, linear_u0=True)
    np.testing.assert_allclose(u0, arr["bratu24_linear_u0"], rtol=1e-13)
    out, rec, so, exc = _run(O.gauss_newton_krylow, prob.make_res(y), u0, prob.make_jac(), max_iter=100)
    case = meta["cases"]["bratu24_linear_res_old"]
    assert so == case["stdout"]
    assert exc is not None and exc[0] == "StepLengthConvergenceError"


def test_bratu24_linear_res_new(golden):
    meta, _ = golden
    prob, y, u0 = O.bratu_workload(24, lam=0.0, linear_u0=True)
    out, rec, so, exc = _run(O.gauss_newton_krylow, prob.make_res(y), u0, prob.make_jac(),
                             version="res_new", max_iter=200)
    _check(meta["cases"]["bratu24_linear_res_new"], out, rec, so, exc, rtol=1e-8)


@pytest.mark.parametrize("version", ["res_old", "res_new"])
@pytest.mark.parametrize("restart", [None, 20])
def test_bratu100_gnk(golden, version, restart):
    meta, arr = golden
    prob, y, u0 = O.bratu_workload(100)
    np.testing.assert_array_equal(u0, arr["bratu100_u0"])
    out, rec, so, exc = _run(O.gauss_newton_krylow, prob.make_res(y), u0, prob.make_jac(),
                             version=version, krylow_restart=restart, max_iter=100)
    _check(meta["cases"][f"bratu100_{version}_r{restart}"], out, rec, so, exc, rtol=1e-9 if restart else RTOL)


@pytest.mark.parametrize("name,kw", [("bratu24_gn", {}), ("bratu24_gn_precond", {"cg_preconditioner": True})])
def test_bratu24_gn(golden, name, kw):
    meta, _ = golden
    prob, y, u0 = O.bratu_workload(24)
    out, rec, so, exc = _run(O.gauss_newton, prob.make_res(y), u0, prob.make_jac(), **kw)
    _check(meta["cases"][name], out, rec, so, exc, rtol=1e-9)


@pytest.mark.parametrize("N", [24, 100])
@pytest.mark.parametrize("pre", [False, True])
def test_cgls_first_step(golden, N, pre):
    meta, arr = golden
    prob, y, u0 = O.bratu_workload(N)
    r0 = prob.make_res(y)(u0)
    J0 = prob.make_jac()(u0)
    x, it = O.cg_least_squares(-1 * J0, r0, preconditioner=pre)
    assert it == meta["cases"][f"cgls{N}_pre{int(pre)}"]["cg_iter"]
    np.testing.assert_allclose(x, arr[f"cgls{N}_pre{int(pre)}__x"], rtol=1e-9, atol=1e-12 * np.abs(x).max())


@pytest.mark.parametrize("N", [8, 64])
def test_single_operators(golden, N):
    meta, arr = golden
    prob = O.BratuPdeProblem(N + 1, 5, 10)
    st = prob.stencil
    u, v, w = arr[f"ops{N}_u"], arr[f"ops{N}_v"], arr[f"ops{N}_w"]
    np.testing.assert_allclose(prob.u_true, arr[f"ops{N}_utrue"], rtol=0, atol=0)
    np.testing.assert_allclose(st.jvp(u, v), arr[f"ops{N}_Jv"], rtol=1e-14, atol=1e-14 * np.abs(arr[f"ops{N}_Jv"]).max())
    np.testing.assert_allclose(st.vjp(u, w), arr[f"ops{N}_JTw"], rtol=1e-14, atol=1e-14 * np.abs(arr[f"ops{N}_JTw"]).max())
    np.testing.assert_allclose(st.pde_operator(u), arr[f"ops{N}_F"], rtol=1e-14, atol=1e-14 * np.abs(arr[f"ops{N}_F"]).max())
    np.testing.assert_allclose(st.diag_jtj(u), arr[f"ops{N}_diagJTJ"], rtol=1e-14)
    J = prob.make_jac()(u)
    kr = O.KrylovBasis()
    kr.start(u)
    for step in range(3):
        kr.update(J, arr[f"ops{N}_update_res"][step])
    np.testing.assert_allclose(kr.basis, arr[f"ops{N}_basis"], rtol=1e-12, atol=1e-13)
    JV = J @ kr.basis
    d = O.linear_least_squares(-1 * JV, arr[f"ops{N}_lls_r"])
    np.testing.assert_allclose(d, arr[f"ops{N}_lls_d"], rtol=1e-12)
