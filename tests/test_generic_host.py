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
