"""Operator Jacobians and the device ``Problem(residual, jvp, vjp)``, on CPU.

  * ``jac(x)`` returning a ``scipy.sparse.linalg.LinearOperator`` -- the reference's duck typing: it uses
    jac only through ``@`` / ``.T @`` (ref:gauss_newton_krylow.py:86, ref:krylow.py:62,
    ref:armijo_goldstein.py:50).  The reference itself run with ``aslinearoperator`` (tests/golden/
    operator.json, tests/golden/make_golden_operator.py) reproduces its sparse runs exactly; the device
    solver must reproduce them too (bookkeeping exact, ||x_k|| within 1e-9 as the p = 1000 pin).  For
    gauss_newton the reference raises on an operator (its lstsq branch); this build takes the CGLS
    branch and must reproduce the reference's SPARSE GN run (cg_iter included).
  * a Bratu ``Problem`` written in torch (tests/torch_bratu.py) reproduces the reference's Bratu runs
    and the matrix-free Bratu path (1e-10), with explicit and with autodiff (torch.func) products.

Checks are shared with tests/test_gpu_problem.py (backend {} = the HIP library).
"""
import contextlib
import io
import json
import os

import numpy as np
import pytest
import scipy.sparse
import scipy.sparse.linalg
import torch

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
from oracle import gnk_oracle as O
from tests.numpy_backend import NumpyBackend
from tests.test_generic_host import rosen_x0
from tests.test_oracle_golden import _check, _run
from tests.torch_bratu import make_torch_bratu

OPERATOR_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "operator.json")


def operator_golden():
    with open(OPERATOR_GOLDEN) as f:
        return json.load(f)


def op_jac(jac):
    return lambda x: scipy.sparse.linalg.aslinearoperator(jac(x))


def check_operator_gnk(golden, x0name, version, backend_kw):
    meta, arr = golden
    opg = operator_golden()["cases"][f"rosen1000_{x0name}_{version}_op"]
    assert opg["same_as_sparse"]                       # the reference: operator run == sparse run
    res, jac = O.rosenbrock(1000)
    x0 = rosen_x0(arr, 1000, x0name)
    out, rec, so, exc = _run(gnk.gauss_newton_krylow, res, x0, op_jac(jac), version=version, **backend_kw)
    assert (out.nit, out.nrev, out.njev, out.success) == (opg["nit"], opg["nrev"], opg["njev"], opg["success"])
    assert so == opg["stdout"] and rec["nfev"] == opg["per_iter"]["nfev"]
    np.testing.assert_allclose(rec["xnorm"], opg["per_iter"]["xnorm"], rtol=1e-9)
    if version in ("res_old", "res_new"):
        _check(meta["cases"][f"rosen1000_{x0name}_{version}"], out, rec, so, exc, rtol=1e-9)


def check_operator_gn(golden, x0name, backend_kw):
    """The reference raises for an operator in gauss_newton (recorded); the device takes CGLS and reproduces
    the reference's sparse-Jacobian run: cg_iter per iteration, nfev, stdout exact."""
    meta, arr = golden
    opg = operator_golden()["cases"][f"rosen1000_{x0name}_gn_op"]
    assert opg["exception"][0] == "ValueError"
    res, jac = O.rosenbrock(1000)
    x0 = rosen_x0(arr, 1000, x0name)
    out, rec, so, exc = _run(gnk.gauss_newton, res, x0, op_jac(jac), **backend_kw)
    _check(meta["cases"][f"rosen1000_{x0name}_gn"], out, rec, so, exc, rtol=1e-9)


@pytest.mark.parametrize("x0name", ["i", "ii", "iii"])
@pytest.mark.parametrize("version", ["res_old", "res_new", "jac_old_res_old", "jac_old_res_new"])
def test_operator_jacobian_gnk(golden, x0name, version):
    check_operator_gnk(golden, x0name, version, dict(_backend=NumpyBackend()))


@pytest.mark.parametrize("x0name", ["i", "iii"])
def test_operator_jacobian_gn_takes_cgls(golden, x0name):
    check_operator_gn(golden, x0name, dict(_backend=NumpyBackend()))


def test_plain_object_operator():
    """Any object with ``@`` and ``.T`` (no scipy base class) is an operator Jacobian."""
    res, jac = O.rosenbrock(2)

    class Op:
        def __init__(self, A):
            self.A = A

        def __matmul__(self, v):
            return self.A @ v

        @property
        def T(self):
            return Op(self.A.T)

    a = gnk.gauss_newton_krylow(res, np.array([2.0, 2.0]), lambda x: Op(jac(x).toarray()), _backend=NumpyBackend())
    b = O.gauss_newton_krylow(res, np.array([2.0, 2.0]), jac)
    assert (a.nit, a.nrev, a.njev, a.success) == (b.nit, b.nrev, b.njev, b.success)
    np.testing.assert_allclose(a.x, b.x, rtol=1e-12)


# -- device Problem ------------------------------------------------------------------------------------
def bratu_problem(N, y, autodiff=False, with_diag=True, lam=10.0, alpha=5.0, grid_resolution=None):
    r, jv, vj, dg = make_torch_bratu(N, alpha, lam, y, grid_resolution, with_jvp=not autodiff, with_diag=with_diag)
    return gnk.Problem(r, jv, vj, diag_jtj=dg)


def run_problem(method, prob, u0, backend_kw, **kw):
    rec = {"xnorm": [], "rnorm": [], "nfev": [], "cg_iter": []}
    res = prob.make_res()

    def cb(x, nfev, cg_iter):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(res(x))))
        rec["nfev"].append(nfev)
        rec["cg_iter"].append(cg_iter)

    buf, exc, out = io.StringIO(), None, None
    with contextlib.redirect_stdout(buf):
        try:
            out = method(res, u0, prob.make_jac(), callback=cb, **backend_kw, **kw)
        except gnk.StepLengthConvergenceError as e:
            exc = ["StepLengthConvergenceError", e.message]
    return out, rec, buf.getvalue().splitlines(), exc


def check_problem_bratu24(golden, name, kw, backend_kw, autodiff=False, with_diag=True):
    """A torch Bratu Problem at N = 24 against the reference's golden run ``name`` (1e-10)."""
    meta, arr = golden
    prob = bratu_problem(24, arr["bratu24_y"], autodiff=autodiff, with_diag=with_diag)
    method = gnk.gauss_newton if name.endswith(("_gn", "_gn_precond")) else gnk.gauss_newton_krylow
    out, rec, so, exc = run_problem(method, prob, arr["bratu24_u0"], backend_kw, **kw)
    case = meta["cases"][name]
    assert so == case["stdout"] and exc == case["exception"]
    assert (out.nit, out.nrev, out.njev, out.success) == (case["nit"], case["nrev"], case["njev"], case["success"])
    assert rec["nfev"] == case["per_iter"]["nfev"] and rec["cg_iter"] == case["per_iter"]["cg_iter"]
    np.testing.assert_allclose(rec["xnorm"], case["per_iter"]["xnorm"], rtol=1e-10)
    np.testing.assert_allclose(rec["rnorm"], case["per_iter"]["rnorm"], rtol=1e-10,
                               atol=1e-10 * case["per_iter"]["rnorm"][0])


@pytest.mark.parametrize("name,kw", [("bratu24_res_old_rNone", dict(version="res_old", max_iter=100)),
                                     ("bratu24_res_new_rNone", dict(version="res_new", max_iter=100)),
                                     ("bratu24_jac_old_res_old_rNone", dict(version="jac_old_res_old", max_iter=100)),
                                     ("bratu24_gn", {}), ("bratu24_gn_precond", dict(cg_preconditioner=True))])
def test_problem_bratu24(golden, name, kw):
    check_problem_bratu24(golden, name, kw, dict(_backend=NumpyBackend()))


def test_problem_autodiff_and_probed_diagonal(golden):
    """Problem(residual) alone: J v and J^T w by torch.func, diag(J^T J) probed with unit vectors."""
    check_problem_bratu24(golden, "bratu24_res_new_rNone", dict(version="res_new", max_iter=100),
                          dict(_backend=NumpyBackend()), autodiff=True)
    check_problem_bratu24(golden, "bratu24_gn", {}, dict(_backend=NumpyBackend()), autodiff=True, with_diag=False)


def test_problem_callables_drop_into_host_code(golden):
    """make_res() / make_jac() as the reference's closures: NumPy in, NumPy out; J @ V on (n, k), J.T @ w,
    -1 * J; the oracle's own (reference-restating) solver runs on them."""
    meta, arr = golden
    y, u0 = arr["bratu24_y"], arr["bratu24_u0"]
    prob = bratu_problem(24, y)
    ref_prob = O.BratuPdeProblem(25, 5, 10)
    res, jac = prob.make_res(), prob.make_jac()
    J, Jr = jac(u0), ref_prob.make_jac()(u0)
    rng = np.random.default_rng(0)
    V, w = rng.standard_normal((576, 3)), rng.standard_normal(576)
    np.testing.assert_allclose(res(u0), ref_prob.make_res(y)(u0), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(J @ V, Jr @ V, rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose((-1 * J).T @ w, -(Jr.T @ w), rtol=1e-12, atol=1e-9)
    p2 = gnk.BratuPdeProblem(25, 5, 10)                  # the reference's CSR assembly (compat views)
    Jcsr = -1 * (p2.laplace2d + 5 * p2.partial_diff_x + 10 * scipy.sparse.diags(np.exp(u0)))
    np.testing.assert_allclose(J.diagonal_ata(), (Jcsr.T @ Jcsr).diagonal(), rtol=1e-13)
    assert J.shape == (576, 576) and torch.is_tensor(J @ torch.as_tensor(w))
    with contextlib.redirect_stdout(io.StringIO()):
        a = O.gauss_newton_krylow(res, u0, jac, max_iter=20)
        b = O.gauss_newton_krylow(ref_prob.make_res(y), u0, ref_prob.make_jac(), max_iter=20)
    assert (a.nit, a.nrev, a.njev) == (b.nit, b.nrev, b.njev)
    np.testing.assert_allclose(a.x, b.x, rtol=1e-9)


def test_problem_args_and_shorthand():
    """res(x, *args) -> residual(x, *args) etc.; ``gauss_newton_krylow(problem, x0, None)``."""
    A = torch.as_tensor(np.array([[1.0, 2.0], [3.0, 1.0], [0.5, -1.0]]))
    y = torch.as_tensor(np.array([1.0, 2.0, 0.5]))
    prob = gnk.Problem(lambda x, s: s * (y - A @ x) + 0.1 * torch.sin(x).sum())
    ref_res = lambda x: (y - A @ torch.as_tensor(x)).numpy() + 0.1 * np.sin(x).sum()  # noqa: E731
    ref_jac = lambda x: -A.numpy() + 0.1 * np.cos(x)[None, :] * np.ones((3, 1))  # noqa: E731
    x0 = np.array([0.5, -0.5])
    with contextlib.redirect_stdout(io.StringIO()):
        a = gnk.gauss_newton_krylow(prob.make_res(), x0, prob.make_jac(), args=(1.0,), _backend=NumpyBackend())
        c = O.gauss_newton_krylow(ref_res, x0, ref_jac)
        d = gnk.gauss_newton_krylow(gnk.Problem(lambda x: y - A @ x + 0.1 * torch.sin(x).sum()), x0, None,
                                    _backend=NumpyBackend())
    # (the converged last step's Armijo count is a rounding tie at this size: nrev is not compared)
    assert (a.nit, a.nrev, a.njev) == (d.nit, d.nrev, d.njev)
    np.testing.assert_array_equal(a.x, d.x)
    assert (a.nit, a.njev, a.success) == (c.nit, c.njev, c.success)
    np.testing.assert_allclose(a.x, c.x, rtol=1e-8)
    with pytest.raises(TypeError):
        gnk.gauss_newton_krylow(prob.make_res(), x0, lambda x: None, _backend=NumpyBackend())
