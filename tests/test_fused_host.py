"""Host logic of the fused first trial + next Gram pass, on the NumPy double of the
C-ABI (tests/numpy_backend.py) -- no GPU.

* gnk_lls_proj's Gram-space projection == the Gram of the materialised column (gnk_lls_next's T);
* GNK res_old with the fused pass on every eligible step (FUSED_KMIN lowered) follows the unfused
  solver and the oracle (the reference's algorithm): bookkeeping, messages and nfev exact, ||x_k||
  at 1e-10; on one rank and on 2 slab ranks (gloo);
* a rejected Gram-space projection (rho^2 below RHO2_MIN) falls back to a pass over the materialised
  column and leaves the trajectory unchanged.
"""
import contextlib
import io
import importlib

import numpy as np
import pytest
import torch

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
from gauss_newton_via_generalized_krylov_subspaces_amd import lls as lls_mod
from oracle import gnk_oracle as O
from tests.numpy_backend import NumpyBackend

gnk_mod = importlib.import_module("gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton_krylow")


def _run(N, fused, kmin=3, max_iter=40, version="res_old", comm=None, rho2=None):
    prob_o, y, u0 = O.bratu_workload(N)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    res_o = prob_o.make_res(y)
    xs, rs, nf = [], [], []
    old = (gnk_mod.BratuOps.fused_kmin, lls_mod.RHO2_MIN, gnk_mod.GNKSolver.FUSED_DEFAULT)
    gnk_mod.BratuOps.fused_kmin = kmin if fused else 10 ** 9
    gnk_mod.GNKSolver.FUSED_DEFAULT = True
    if rho2 is not None:
        lls_mod.RHO2_MIN = rho2
    solver_ref = {}
    init = gnk_mod.GNKSolver.__init__

    def init_spy(self, *a, **k):
        init(self, *a, **k)
        solver_ref["s"] = self

    gnk_mod.GNKSolver.__init__ = init_spy
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            out = gnk.gauss_newton_krylow(prob.make_res(y), u0, prob.make_jac(), krylow_restart=20,
                                          max_iter=max_iter, version=version, comm=comm, _backend=NumpyBackend(),
                                          callback=lambda x, nfev, cg_iter: (xs.append(np.linalg.norm(x)),
                                                                             rs.append(np.linalg.norm(res_o(x))),
                                                                             nf.append(nfev)))
    finally:
        gnk_mod.GNKSolver.__init__ = init
        gnk_mod.BratuOps.fused_kmin, lls_mod.RHO2_MIN, gnk_mod.GNKSolver.FUSED_DEFAULT = old
    return out, np.array(xs), np.array(rs), nf, buf.getvalue(), solver_ref["s"]


def _oracle(N, max_iter=40, version="res_old"):
    prob_o, y, u0 = O.bratu_workload(N)
    res_o = prob_o.make_res(y)
    xs, nf = [], []
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = O.gauss_newton_krylow(res_o, u0, prob_o.make_jac(), krylow_restart=20, max_iter=max_iter,
                                    version=version, callback=lambda x, nfev, cg_iter: (xs.append(np.linalg.norm(x)),
                                                                                         nf.append(nfev)))
    return out, np.array(xs), nf, buf.getvalue()


def test_lls_proj_matches_materialised_gram():
    """Gram-space projection of the fused Gram == the Gram over the materialised pending column."""
    rng = np.random.default_rng(3)
    be = NumpyBackend()
    N = 128
    be.set_bratu(N, 0, N, 1.0 / (N + 1), 5.0, 10.0)
    n = be.slab_len()
    k = 6                                          # step i: 5 settled + 1 pending (raw)
    V = torch.zeros(k + 2, n, dtype=torch.float64)
    own = slice(2 * N, (2 + N) * N)
    V[:, own] = torch.from_numpy(rng.standard_normal((k + 2, N * N)) / N)
    u = torch.from_numpy(rng.standard_normal(n) * 0.1)
    r = torch.from_numpy(rng.standard_normal(n))
    u[:2 * N] = 0
    u[-2 * N:] = 0
    r[:2 * N] = 0
    r[-2 * N:] = 0
    # a plausible step-i solve: R upper triangular, its inverse in `out`
    R = np.triu(rng.standard_normal((k, k))) + 3 * np.eye(k)
    out = np.zeros(3 + k + 3 * k * k)
    out[3 + k:3 + k + k * k] = R.reshape(-1)
    out[3 + k + 2 * k * k:] = np.linalg.inv(R).reshape(-1)
    out = torch.from_numpy(out)
    etry = torch.from_numpy(rng.standard_normal(k))
    sc = torch.from_numpy(np.abs(rng.standard_normal(k)) + 0.5)
    h = rng.standard_normal(k) * 0.3
    pack = torch.from_numpy(np.concatenate([[0.0, 2.0, 0.0], h]))
    kp = be.gram_dim(k + 1, True)
    # fused: Gram of [J V T_f | J g | r]  (g = V[k] here stands in for the pass's update column)
    Tf = torch.zeros(kp * kp, dtype=torch.float64)
    be.lls_fused_t(k, out, sc, kp, Tf)
    Gf = torch.zeros(kp * kp, dtype=torch.float64)
    be.gram(u, V, k + 1, Tf, r, Gf)
    Gp = torch.zeros(kp * kp, dtype=torch.float64)
    bufs = [torch.zeros(64, dtype=torch.float64) for _ in range(5)]
    P1, sdd1, e1, hh1, sc1 = bufs
    be.lls_proj(k, out, etry, pack, sc, kp, Gf, 0.0, Gp, P1, sdd1, e1, hh1, sc1)
    # reference: gnk_lls_next's T (with -hh in the pending column) over the same V
    T2 = torch.zeros(kp * kp, dtype=torch.float64)
    P2, sdd2, e2, hh2, sc2 = [torch.zeros(64, dtype=torch.float64) for _ in range(5)]
    be.lls_next(k, True, out, etry, pack, sc, kp, T2, P2, sdd2, e2, hh2, sc2)
    # T2's row k-1 carries (1/nrm) * nrm: equal to T_f's 1 up to rounding
    G2 = torch.zeros(kp * kp, dtype=torch.float64)
    be.gram(u, V, k + 1, T2, r, G2)
    a, b = Gp.numpy().reshape(kp, kp)[:k + 2, :k + 2], G2.numpy().reshape(kp, kp)[:k + 2, :k + 2]
    np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-11 * np.abs(b).max())
    for x1, x2 in ((P1, P2), (sdd1, sdd2), (e1, e2), (hh1, hh2), (sc1, sc2)):
        np.testing.assert_array_equal(x1.numpy(), x2.numpy())


@pytest.mark.parametrize("N", [128, 256])
def test_fused_gnk_matches_unfused_and_oracle(N):
    out_f, xf, rf, nf_f, so_f, sf = _run(N, True)
    out_u, xu, ru, nf_u, so_u, su = _run(N, False)
    out_o, xo, nf_o, so_o = _oracle(N)
    assert sf.fused_stats["passes"] > 10 and su.fused_stats["passes"] == 0
    assert sf.fused_stats["fallback"] <= sf.fused_stats["passes"] // 4     # rho^2 < RHO2_MIN: small k only
    assert so_f == so_u == so_o
    assert nf_f == nf_u == nf_o
    assert (out_f.nit, out_f.nrev, out_f.njev, out_f.success) == (out_o.nit, out_o.nrev, out_o.njev, out_o.success)
    assert sf.spec_stats["hit"] >= su.spec_stats["hit"] - 1
    # the first restart cycle agrees to rounding; after the res_old restart the trajectory amplifies
    # rounding (tests/golden/sensitivity.json): fused and unfused both stay within 1e-10 of the oracle
    np.testing.assert_allclose(xf[1:21], xo[1:21], rtol=1e-11)   # k = 1 cancels (sensitivity.json)
    np.testing.assert_allclose(xf, xo, rtol=1e-10)
    np.testing.assert_allclose(xf, xu, rtol=1e-10)
    np.testing.assert_allclose(out_f.x, out_u.x, rtol=0, atol=1e-9 * np.abs(out_u.x).max())


def test_fused_projection_fallback_keeps_trajectory():
    """rho^2 threshold above 1: every Gram-space projection is rejected -> the host re-runs the pass on
    the materialised column; the trajectory is the unfused one."""
    out_f, xf, rf, nf_f, so_f, sf = _run(128, True, rho2=2.0)
    out_u, xu, ru, nf_u, so_u, su = _run(128, False)
    assert sf.fused_stats["passes"] > 10
    assert sf.fused_stats["fallback"] > 0
    assert so_f == so_u and nf_f == nf_u
    np.testing.assert_allclose(xf, xu, rtol=1e-10)
