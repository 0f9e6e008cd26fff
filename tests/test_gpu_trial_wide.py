"""The wide fused first trial (k_trial_w, 25..208 basis columns) on the GPU.

gnk_basis_gemv_vjp_gemv_t(_pending) with more than 24 columns materialises the pending column w = g - V hh, forms
x = V c, g = -J(x)^T r and h = V^T g from one read of V (64-point tiles through LDS).  Checked against fp64 NumPy of
the same quantities and against the unfused kernels (gnk_basis_gemv_pending + gnk_vjp_gemv_t, the path it
replaces; ref:krylow.py:62-64, ref:armijo_goldstein.py:56); then a GNK run whose basis grows past 24 columns
(no restart) against the same run with the fused trial capped at 24 columns: bookkeeping exact, ||x_k|| 1e-10.
"""
import contextlib
import io

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402
from oracle import gnk_oracle as O  # noqa: E402


@pytest.mark.parametrize("N,k,pend", [(512, 25, True), (512, 32, False), (1024, 33, True), (512, 56, True),
                                      (512, 57, True), (256, 100, True), (256, 104, False), (256, 150, True),
                                      (128, 207, True), (128, 208, False)])
def test_trial_wide_matches_numpy_and_unfused(N, k, pend):
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    dev = BratuDevice(prob, Comm(single=True))
    be, sl = dev.backend, dev.slab
    rng = np.random.default_rng(N + k)
    n = N * N
    kk = k + (1 if pend else 0)
    Vh = rng.standard_normal((kk, n)) / np.sqrt(n)
    c = rng.standard_normal(kk)
    hh = 0.1 * rng.standard_normal(k)
    rh = rng.standard_normal(n)
    V = be.zeros(kk, sl.length)
    for j in range(kk):
        V[j].copy_(dev.load(Vh[j]))
    r = dev.load(rh)
    cd, hd = be.to_device(c), be.to_device(hh)
    outs = {}
    for mode in ("wide", "unfused"):
        Vm = V.clone()
        x, g, h, st = dev.vec(), dev.vec(), be.zeros(kk), be.zeros(4)
        if mode == "wide":
            if pend:
                be.gemv_vjp_gemv_t_pending(Vm, k, cd, hd, r, x, g, h, st)
            else:
                be.gemv_vjp_gemv_t(Vm, kk, cd, r, x, g, h)
        else:
            if pend:
                be.gemv_pending(Vm, k, cd, hd, x, st)
            else:
                be.gemv(Vm, kk, cd, x)
            be.vjp_gemv_t(x, r, Vm, kk, g, h)
        torch.cuda.synchronize()
        outs[mode] = {"x": x[sl.own].cpu().numpy(), "g": g[sl.own].cpu().numpy(), "h": h.cpu().numpy(),
                      "w": Vm[min(k, kk - 1)][sl.own].cpu().numpy(), "st": st[:2].cpu().numpy()}
    a, b = outs["wide"], outs["unfused"]
    # fp64 NumPy of the same products
    W = Vh.copy()
    if pend:
        W[k] = Vh[k] - hh @ Vh[:k]
    xr = c @ W
    op = O.BratuPdeProblem(N + 1, 5, 10)
    gr = -(op.make_jac()(xr).T @ rh)
    hr = W @ gr
    sx = np.abs(W).T @ np.abs(c)
    np.testing.assert_allclose(a["x"], xr, rtol=0, atol=1e-13 * sx.max())
    np.testing.assert_allclose(a["x"], b["x"], rtol=0, atol=1e-13 * sx.max())
    np.testing.assert_allclose(a["g"], b["g"], rtol=1e-12, atol=1e-12 * np.abs(gr).max())
    np.testing.assert_allclose(a["h"], hr, rtol=1e-10, atol=1e-12 * np.abs(W).sum(1).max() * np.abs(gr).max())
    np.testing.assert_allclose(a["h"], b["h"], rtol=1e-10, atol=1e-12 * np.abs(W).sum(1).max() * np.abs(gr).max())
    if pend:
        np.testing.assert_allclose(a["w"], W[k], rtol=0, atol=1e-14 * np.abs(W[k]).max() * 10)
        np.testing.assert_allclose(a["st"][0], np.sum(W[k] ** 2), rtol=1e-12)
        assert a["st"][1] == np.max(np.abs(a["w"]))


def _gnk_run(N, fuse_kmax, max_iter):
    _, y, u0 = O.bratu_workload(N)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    s = gnk.GNKSolver(prob, y, krylow_restart=None, max_iter=max_iter, version="res_old")
    if fuse_kmax is not None:
        s.basis.FUSE_KMAX = fuse_kmax
    rec = []
    s.callback = lambda x, nfev, cg_iter: rec.append((float(np.linalg.norm(x)), nfev))
    with contextlib.redirect_stdout(io.StringIO()):
        s.setup(u0)
        while not s.step():
            pass
        out = s.finish()
    return out, rec


def test_gnk_wide_fused_trial_matches_unfused():
    """N = 256, no restart, 45 iterations (k to 44): the fused wide trial from k = 25 against the unfused path."""
    a, ra = _gnk_run(256, None, 45)
    b, rb = _gnk_run(256, 24, 45)
    assert (a.nit, a.nrev, a.njev, a.success) == (b.nit, b.nrev, b.njev, b.success)
    assert [n for _, n in ra] == [n for _, n in rb]
    np.testing.assert_allclose([v for v, _ in ra], [v for v, _ in rb], rtol=1e-10)
