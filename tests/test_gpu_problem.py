"""Operator Jacobians and the device ``Problem`` on the GPU (checks of
tests/test_problem_operator.py with the HIP library as the backend).

  * Rosenbrock p = 1000 (F5) with ``jac`` wrapped in ``aslinearoperator``: GNK in all four versions against
    the reference's own operator runs (tests/golden/operator.json) and GN against its sparse run;
  * a torch Bratu ``Problem`` at N = 24 against the reference's golden runs, and at N = 100 against the
    matrix-free Bratu path of this package (the reference's F3 workload, no restart, 1e-10).
"""
import contextlib
import io

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from oracle import gnk_oracle as O  # noqa: E402
from tests.test_problem_operator import (bratu_problem, check_operator_gn, check_operator_gnk,  # noqa: E402
                                         check_problem_bratu24, run_problem)


@pytest.mark.parametrize("x0name", ["i", "ii", "iii"])
@pytest.mark.parametrize("version", ["res_old", "res_new", "jac_old_res_old", "jac_old_res_new"])
def test_gpu_operator_jacobian_gnk(golden, x0name, version):
    check_operator_gnk(golden, x0name, version, {})


@pytest.mark.parametrize("x0name", ["i", "ii", "iii"])
def test_gpu_operator_jacobian_gn_takes_cgls(golden, x0name):
    check_operator_gn(golden, x0name, {})


@pytest.mark.parametrize("name,kw", [("bratu24_res_old_rNone", dict(version="res_old", max_iter=100)),
                                     ("bratu24_res_new_rNone", dict(version="res_new", max_iter=100)),
                                     ("bratu24_jac_old_res_new_rNone", dict(version="jac_old_res_new", max_iter=100)),
                                     ("bratu24_gn", {}), ("bratu24_gn_precond", dict(cg_preconditioner=True))])
def test_gpu_problem_bratu24(golden, name, kw):
    check_problem_bratu24(golden, name, kw, {})


def test_gpu_problem_autodiff(golden):
    check_problem_bratu24(golden, "bratu24_res_old_rNone", dict(version="res_old", max_iter=100), {}, autodiff=True)


@pytest.mark.parametrize("version", ["res_old", "res_new"])
def test_gpu_problem_bratu100_matches_matrix_free(version):
    """N = 100 (grid 101, the reference's compare() workload), no restart (k grows to 99: the flat Gram's
    MFMA tiles to 63 columns, the wide pass beyond): the torch Problem's trajectory equals the matrix-free
    Bratu path's -- bookkeeping exact, ||x_k|| and ||r_k|| within 1e-10 at every iteration."""
    _, y, u0 = O.bratu_workload(100)
    prob = bratu_problem(100, y)
    a = run_problem(gnk.gauss_newton_krylow, prob, u0, {}, version=version, max_iter=100)
    bp = gnk.BratuPdeProblem(101, 5, 10)
    rec = {"xnorm": [], "rnorm": [], "nfev": []}
    ref_res = prob.make_res()

    def cb(x, nfev, cg_iter):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(ref_res(x))))
        rec["nfev"].append(nfev)

    with contextlib.redirect_stdout(io.StringIO()):
        b = gnk.gauss_newton_krylow(bp.make_res(y), u0, bp.make_jac(), version=version, max_iter=100, callback=cb)
    out, ra = a[0], a[1]
    assert (out.nit, out.nrev, out.njev, out.success) == (b.nit, b.nrev, b.njev, b.success)
    assert ra["nfev"] == rec["nfev"]
    np.testing.assert_allclose(ra["xnorm"], rec["xnorm"], rtol=1e-10)
    np.testing.assert_allclose(ra["rnorm"], rec["rnorm"], rtol=1e-10)


def test_gpu_problem_stays_on_device():
    """The Problem's callables see device tensors of the solver's device (no host round trip)."""
    _, y, u0 = O.bratu_workload(24)
    r, jv, vj, dg = __import__("tests.torch_bratu", fromlist=["x"]).make_torch_bratu(24, 5.0, 10.0, y)
    seen = set()

    def res(x):
        seen.add((x.device.type, x.dtype))
        return r(x)

    with contextlib.redirect_stdout(io.StringIO()):
        gnk.gauss_newton_krylow(gnk.Problem(res, jv, vj), u0, None, max_iter=5)
    assert seen == {("cuda", torch.float64)}
