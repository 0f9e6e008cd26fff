"""An adopted speculative solve's device-formed coefficients: the first trial takes the
pending column's projection hh' and the next speculation takes the column scales sc' from the buffers
k_lls_next wrote, instead of uploading the host's copies.  The host computes the same values from the
same inputs with the same IEEE operations, so the run must be bit for bit the run that uploads them
(C2's workload: N = 1024, restart 20, res_old; ref:gauss_newton_krylow.py:84-136, ref:krylow.py:62-73)."""
import contextlib
import io

import numpy as np
import pytest

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
from gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton_krylow import GNKSolver
from oracle import gnk_oracle as O

pytestmark = pytest.mark.gpu


def _run(reuse, N=1024, max_iter=45):
    _, y, u0 = O.bratu_workload(N)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    rec = []
    old = GNKSolver.reuse_spec_device
    GNKSolver.reuse_spec_device = reuse
    try:
        with contextlib.redirect_stdout(io.StringIO()) as out:
            res = gnk.gauss_newton_krylow(prob.make_res(y), u0, prob.make_jac(), krylow_restart=20, max_iter=max_iter,
                                          callback=lambda x, nfev, cg_iter: rec.append((float(np.dot(x, x)), nfev)))
    finally:
        GNKSolver.reuse_spec_device = old
    return rec, (res.nit, res.nfev, res.njev), out.getvalue(), res.x


def test_spec_device_coefficients_bit_identical():
    a, ba, sa, xa = _run(True)
    b, bb, sb, xb = _run(False)
    assert ba == bb and sa == sb
    assert [n for _, n in a] == [n for _, n in b]
    assert [v for v, _ in a] == [v for v, _ in b]          # ||x_k||^2 of every iterate, exactly
    assert np.array_equal(xa, xb)
