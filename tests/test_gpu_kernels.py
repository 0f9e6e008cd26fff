"""HIP kernels (through the C-ABI) against the CPU oracle / exact NumPy restatements.

Tolerances: stencil kernels follow scipy's CSR summation order with
-ffp-contract=off, so they agree with the oracle to a few ulps (checked at
1e-13 relative to the operator scale); reductions differ only in summation order.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from gauss_newton_via_generalized_krylov_subspaces_amd import _native  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.bratu_pde_problem import BratuPdeProblem  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402
from oracle import gnk_oracle as O  # noqa: E402

G = _native.GHOST


def make(N, lam=10.0, alpha=5.0):
    prob = BratuPdeProblem(N + 1, alpha, lam)
    dev = BratuDevice(prob, Comm(single=True))
    ref = O.BratuStencil(N, alpha, lam, prob.grid_resolution)
    return prob, dev, ref


def own(dev, t):
    return t[dev.slab.own].cpu().numpy()


def close(a, b, scale=None, rtol=1e-13):
    scale = np.abs(b).max() if scale is None else scale
    np.testing.assert_allclose(a, b, rtol=0, atol=rtol * max(scale, 1e-300))


@pytest.mark.parametrize("N", [8, 25, 64, 512, 1024])     # N % 512 == 0: the two-row k_jvp2 / k_forward2
@pytest.mark.parametrize("lam", [10.0, 0.0])
def test_operators_match_oracle(N, lam):
    prob, dev, ref = make(N, lam)
    rng = np.random.default_rng(N)
    n = N * N
    u = 0.3 * rng.standard_normal(n)
    v = rng.standard_normal(n)
    be = dev.backend
    us, vs = dev.load(u), dev.load(v)
    out = dev.vec()
    be.jvp(us, vs, out)
    close(own(dev, out), ref.jvp(u, v))
    be.vjp(us, vs, out)
    close(own(dev, out), ref.vjp(u, v))
    be.forward(us, out)
    close(own(dev, out), ref.pde_operator(u))
    be.diag_jtj(us, out)
    close(own(dev, out), ref.diag_jtj(u))
    be.diag_jtj(us, out, reciprocal=True)
    np.testing.assert_allclose(own(dev, out), 1.0 / ref.diag_jtj(u), rtol=1e-14)
    y = ref.pde_operator(0.5 * u)
    n2 = dev.scalar(1)
    be.residual(us, dev.load(y), out, n2)
    r_ref = y - ref.pde_operator(u)
    close(own(dev, out), r_ref)
    np.testing.assert_allclose(n2.item(), np.sum(r_ref ** 2), rtol=1e-12)


@pytest.mark.parametrize("N", [64, 512])     # k_jvp (one row per pass) / k_jvp2 (two rows, N % 512 == 0)
def test_jvp_bitwise_vs_oracle_small(N):
    """With the CSR summation order and no FMA contraction the stencil is bit-exact vs the oracle
    except where exp() differs by an ulp (lambda = 0 removes exp)."""
    prob, dev, ref = make(N, lam=0.0)
    rng = np.random.default_rng(7)
    v = rng.standard_normal(N * N)
    out = dev.vec()
    dev.backend.jvp(dev.load(np.zeros(N * N)), dev.load(v), out)
    np.testing.assert_array_equal(own(dev, out), ref.jvp(np.zeros(N * N), v))
    dev.backend.vjp(dev.load(np.zeros(N * N)), dev.load(v), out)
    np.testing.assert_array_equal(own(dev, out), ref.vjp(np.zeros(N * N), v))
    x = rng.standard_normal(N * N)
    dev.backend.forward(dev.load(x), out)
    close(own(dev, out), ref.pde_operator(x), rtol=1e-14)


@pytest.mark.parametrize("N,k", [(24, 1), (24, 7), (100, 33), (1024, 20), (25, 5), (128, 70), (96, 41)])
def test_basis_kernels(N, k):
    prob, dev, ref = make(N)
    be = dev.backend
    rng = np.random.default_rng(k)
    L = dev.slab.length
    V = be.zeros(k + 1, L)
    Vh = rng.standard_normal((k + 1, N * N))
    for j in range(k + 1):
        V[j].copy_(dev.load(Vh[j]))
    c = rng.standard_normal(k)
    x = dev.vec()
    be.gemv(V, k, be.to_device(c), x)
    np.testing.assert_allclose(own(dev, x), c @ Vh[:k], rtol=1e-12, atol=1e-12 * np.abs(Vh).max() * k)
    u = 0.3 * rng.standard_normal(N * N)
    r = rng.standard_normal(N * N)
    us, rs = dev.load(u), dev.load(r)
    h = be.zeros(k)
    g = V[k]
    be.vjp_gemv_t(us, rs, V, k, g, h)
    g_ref = -ref.vjp(u, r)
    close(own(dev, g), g_ref)
    np.testing.assert_allclose(h.cpu().numpy(), Vh[:k] @ g_ref, rtol=1e-11, atol=1e-11 * np.abs(g_ref).sum())
    hh = rng.standard_normal(k)
    st = be.zeros(2)
    be.cgs_update(V, k, be.to_device(hh), g, st)
    g2 = g_ref - hh @ Vh[:k]
    np.testing.assert_allclose(own(dev, g), g2, rtol=1e-12, atol=1e-12 * np.abs(g2).max() * k)
    np.testing.assert_allclose(st[0].item(), np.sum(g2 ** 2), rtol=1e-12)
    assert st[1].item() == np.abs(own(dev, g)).max()
    be.vec_stats(g, st)
    np.testing.assert_allclose(st[0].item(), np.sum(own(dev, g) ** 2), rtol=1e-13)
    be.vec_div(g, 3.0, x, False)
    np.testing.assert_array_equal(own(dev, x), own(dev, g) / 3.0)
    be.vec_axpy(us, 0.25, rs, x, True)
    np.testing.assert_array_equal(own(dev, x), u + 0.25 * r)


@pytest.mark.parametrize("N,k", [(24, 1), (25, 7), (100, 13), (1024, 20), (1023, 24), (64, 17)])
def test_gemv_vjp_gemv_t_fused(N, k):
    """One read of V: x = V c (whole slab), g = -J(x)^T r, h = V^T g == gemv then vjp_gemv_t(u = x):
    x and g bit for bit (same per-element arithmetic), h within reduction-order rounding."""
    prob, dev, ref = make(N)
    be = dev.backend
    rng = np.random.default_rng(k)
    V = be.zeros(k, dev.slab.length)
    Vh = rng.standard_normal((k, N * N)) / N
    for j in range(k):
        V[j].copy_(dev.load(Vh[j]))
    c = be.to_device(rng.standard_normal(k))
    rs = dev.load(rng.standard_normal(N * N))
    x1, g1, h1 = dev.vec(), dev.vec(), be.zeros(k)
    x2, g2, h2 = dev.vec(), dev.vec(), be.zeros(k)
    be.gemv(V, k, c, x1)
    be.vjp_gemv_t(x1, rs, V, k, g1, h1)
    be.gemv_vjp_gemv_t(V, k, c, rs, x2, g2, h2)
    np.testing.assert_array_equal(x2.cpu().numpy() + 0.0, x1.cpu().numpy() + 0.0)
    np.testing.assert_array_equal(own(dev, g2), own(dev, g1))
    np.testing.assert_allclose(h2.cpu().numpy(), h1.cpu().numpy(), rtol=1e-12,
                               atol=1e-12 * np.abs(own(dev, g1)).sum() * np.abs(Vh).max())


def _pending_case(N, k, seed):
    """A basis of k columns with a raw pending column g at slot k (ghost rows filled as after a
    halo, i.e. whole-slab values), coefficients c (k + 1) and projection coefficients hh."""
    prob, dev, ref = make(N)
    be = dev.backend
    rng = np.random.default_rng(seed)
    V = be.zeros(k + 2, dev.slab.length)
    Vh = rng.standard_normal((k + 1, N * N)) / N
    for j in range(k + 1):
        V[j].copy_(dev.load(Vh[j]))
    hh = rng.standard_normal(k) / N
    c = rng.standard_normal(k + 1)
    return prob, dev, ref, be, V, hh, c


@pytest.mark.parametrize("N,k", [(24, 1), (25, 6), (100, 12), (1024, 19), (1023, 23), (64, 16)])
def test_gemv_pending(N, k):
    """Deferred CGS: w = g - V hh materialised in place == gnk_cgs_update's w bit for bit (whole
    slab), x = V c over k + 1 columns == gnk_basis_gemv on the materialised basis bit for bit,
    {sum w^2, max |w|} over owned rows within reduction-order rounding."""
    prob, dev, ref, be, V, hh, c = _pending_case(N, k, 100 + k)
    V2 = V.clone()
    hd, cd = be.to_device(hh), be.to_device(c)
    x1, st1 = dev.vec(), be.zeros(2)
    be.gemv_pending(V, k, cd, hd, x1, st1)
    # reference: explicit CGS over the whole slab (cgs_update covers owned rows: apply it to the
    # slab-sized rows by hand with the same per-element order) + gemv
    wref = V2[k].cpu().numpy().copy()
    s = np.zeros_like(wref)
    Vn = V2.cpu().numpy()
    for j in range(k):
        s = s + Vn[j] * hh[j]
    wref = wref - s
    np.testing.assert_array_equal(V[k].cpu().numpy(), wref)
    st2 = be.zeros(2)
    g2 = V2[k].clone()
    be.cgs_update(V2, k, hd, g2, st2)
    np.testing.assert_array_equal(own(dev, g2), own(dev, V[k]))
    V2[k].copy_(V[k])
    x2 = dev.vec()
    be.gemv(V2, k + 1, cd, x2)
    np.testing.assert_array_equal(x1.cpu().numpy() + 0.0, x2.cpu().numpy() + 0.0)
    w_own = own(dev, V[k])
    np.testing.assert_allclose(st1[0].item(), np.sum(w_own ** 2), rtol=1e-12)
    assert st1[1].item() == np.abs(w_own).max()
    with pytest.raises(RuntimeError, match="alias"):
        be.gemv_pending(V, k, cd, hd, V[k], st1)


@pytest.mark.parametrize("N,k", [(24, 1), (25, 6), (100, 12), (1024, 19), (1023, 23), (64, 16)])
def test_gemv_vjp_gemv_t_pending(N, k):
    """Fused first trial with a pending column == gemv_pending then vjp_gemv_t(u = x) over k + 1
    columns: w, x and g bit for bit, h (k + 1) and the stats within reduction-order rounding."""
    prob, dev, ref, be, V, hh, c = _pending_case(N, k, 200 + k)
    rng = np.random.default_rng(k)
    rs = dev.load(rng.standard_normal(N * N))
    V2 = V.clone()
    hd, cd = be.to_device(hh), be.to_device(c)
    x1, g1, h1, st1 = dev.vec(), dev.vec(), be.zeros(k + 1), be.zeros(2)
    be.gemv_vjp_gemv_t_pending(V, k, cd, hd, rs, x1, g1, h1, st1)
    x2, g2, h2, st2 = dev.vec(), dev.vec(), be.zeros(k + 1), be.zeros(2)
    be.gemv_pending(V2, k, cd, hd, x2, st2)
    be.vjp_gemv_t(x2, rs, V2, k + 1, g2, h2)
    np.testing.assert_array_equal(V[k].cpu().numpy(), V2[k].cpu().numpy())
    np.testing.assert_array_equal(x1.cpu().numpy() + 0.0, x2.cpu().numpy() + 0.0)
    np.testing.assert_array_equal(own(dev, g1), own(dev, g2))
    scale = np.abs(own(dev, g2)).sum() * np.abs(V2[:k + 1].cpu().numpy()).max()
    np.testing.assert_allclose(h1.cpu().numpy(), h2.cpu().numpy(), rtol=1e-12, atol=1e-12 * scale)
    np.testing.assert_allclose(st1.cpu().numpy(), st2.cpu().numpy(), rtol=1e-12)
    with pytest.raises(RuntimeError, match="alias"):
        be.gemv_vjp_gemv_t_pending(V, k, cd, hd, rs, x1, V[k], h1, st1)


@pytest.mark.parametrize("N,lam", [(8, 10.0), (25, 10.0), (64, 0.0), (1024, 10.0), (1023, 10.0)])
def test_normalize_jnorm(N, lam):
    """v = g / denom bit for bit on the whole slab (ghost rows included) and
    sum (J(u) g)^2 within reduction-order rounding (1e-12 relative)."""
    prob, dev, ref = make(N, lam)
    be = dev.backend
    rng = np.random.default_rng(N)
    u = 0.3 * rng.standard_normal(N * N)
    g = dev.load(rng.standard_normal(N * N))
    v = dev.vec()
    jn2 = be.zeros(1)
    be.normalize_jnorm(dev.load(u), g, 3.7, v, jn2)
    np.testing.assert_array_equal(v.cpu().numpy(), g.cpu().numpy() / 3.7)
    jg = ref.jvp(u, own(dev, g))
    np.testing.assert_allclose(jn2.item(), np.sum(jg ** 2), rtol=1e-12)
    with pytest.raises(RuntimeError, match="alias"):
        be.normalize_jnorm(dev.load(u), g, 3.7, g, jn2)


def test_cgs_max_propagates_nan():
    prob, dev, ref = make(24)
    be = dev.backend
    V = be.zeros(2, dev.slab.length)
    g = dev.load(np.where(np.arange(576) == 100, np.nan, 1e-12))
    st = be.zeros(2)
    be.cgs_update(V, 1, be.zeros(1), g, st)
    assert np.isnan(st[1].item()) and np.isnan(st[0].item())


GRAM_CASES = [(24, 1, False, False), (24, 5, True, True), (100, 20, False, False),
                                                  (100, 20, True, True), (64, 47, True, True), (64, 70, True, False),
                                                  (1024, 20, True, True),
                                                  # marching kernel (N % 64 == 0): NB = 1 both passes, NB = 2 pass 1
                                                  (1024, 3, False, False), (1024, 12, True, True), (128, 15, False, True),
                                                  (1024, 25, False, False), (256, 31, False, False),
                                                  # staged kernel: one block, k = 16 with r, tails 1..4
                                                  (256, 16, True, True), (256, 17, True, True), (128, 18, False, True),
                                                  (256, 19, True, False), (1024, 16, True, True), (256, 4, True, True),
                                                  (512, 12, True, True), (384, 9, False, True),
                                                  # VALU kernel (N % 128 == 0, k <= 8 with r)
                                                  (128, 1, True, False), (256, 2, True, True), (384, 3, True, True),
                                                  (256, 5, True, True), (1024, 6, True, True), (640, 7, True, False),
                                                  (1024, 8, True, True), (256, 9, True, True), (128, 9, True, False),
                                                  (640, 7, True, True), (512, 10, True, True),
                                                  # k = 8..12 at more grid sizes (one-point VALU / staged MFMA)
                                                  (256, 11, True, True), (1024, 12, True, True), (640, 10, True, False),
                                                  (128, 12, True, True), (384, 8, True, False),
                                                  # prefetching wide-basis kernel (KP 32..64; partial tail chunks)
                                                  (64, 51, True, True), (64, 40, False, True), (96, 22, True, True),
                                                  (130, 33, True, True), (48, 60, True, True), (24, 30, True, False),
                                                  # NB = 4: flattened order (N % 32 != 0) / down-strip walks crossing strips
                                                  (100, 55, True, True), (96, 50, True, False), (416, 49, True, True),
                                                  # NB = 5..7: k_gram_x (N % 32 == 0; 1..5 strips) / k_gram (N = 100)
                                                  (128, 70, True, True), (96, 90, True, True), (64, 100, True, True),
                                                  (160, 81, False, True), (32, 64, True, True), (100, 75, True, True),
                                                  # k_gram_x plain passes (RinvAug = identity, Gram straight from W)
                                                  (128, 70, True, False), (96, 90, False, False),
                                                  # pair-split k_gram, k >= 112 (C5's range on 8 GPUs)
                                                  (64, 112, True, True), (96, 150, True, False), (64, 200, True, True),
                                                  (32, 130, False, False),
                                                  # two-block Gram at N % 128 != 0 (not the staged kernel), one
                                                  # 128-point strip, without r
                                                  (64, 17, True, True), (192, 20, True, True), (320, 18, False, False),
                                                  (128, 19, False, True), (1024, 18, True, True),
                                                  # k_gram_q's wide instances (k = 21..31, N % 128 == 0, with P^-1)
                                                  (256, 21, True, True), (128, 24, True, True), (256, 27, True, True),
                                                  (128, 29, True, True), (256, 31, True, True), (384, 26, False, True)]


def _staged_modes(N, k):
    # "forced" / "ring5" only where the staged kernel applies (N % 128 == 0, k <= 20).  The 4x4x4-block form
    # (k_gram_q) is the default from k = 8: "noq" runs k_gram_s there instead, "v1" the one-point VALU kernel at
    # k = 8, 9, "valu" / "tm" k_gram_s's two lead-column forms at k = 17..20; "q" forces k_gram_q at k = 5..7
    if N % 128 == 0 and 21 <= k <= 31:
        return ("default", "noq")              # k_gram_q / the chunked k_gram_w
    if N % 128 != 0 or k > 20:
        return ("default",)
    modes = ("default", "forced", "ring5")
    if k >= 8:
        modes += ("noq",)
    if k in (8, 9):
        modes += ("v1",)
    if k >= 17:
        modes += ("valu", "tm")
    if 5 <= k <= 7:
        modes += ("q",)
    return modes


GRAM_PARAMS = [(N, k, r, ri, st) for (N, k, r, ri) in GRAM_CASES for st in _staged_modes(N, k)]


@pytest.mark.parametrize("N,k,with_r,with_rinv,staged", GRAM_PARAMS)
def test_gram_mfma(N, k, with_r, with_rinv, staged):
    """W = [J V | r] @ RinvAug on fp64 MFMA vs an fp64 NumPy Gram (host BLAS).  "forced" runs
    the staged LDS-DMA kernel for every pass it supports (N % 128 == 0, k <= 20) with its default
    4-slot ring (jdiag batched over 4 rows); "ring5" forces the 5-slot ring (one jdiag per row step); "noq" runs
    k_gram_s instead of the 4x4x4-block k_gram_q (default from k = 8), "v1" the one-point VALU kernel at k = 8, 9,
    "valu" / "tm" k_gram_s's lead columns' sums at k = 17..20 on VALU / on 4x4x4 blocks, "q" forces k_gram_q at
    k = 5..7."""
    prob, dev, ref = make(N)
    be = dev.backend
    if staged == "v1":
        be.set_tuning("gram_q", 1)
    elif staged != "default":
        be.set_tuning("gram_path", 1)
        if staged == "ring5":
            be.set_tuning("gram_ring", 5)
        if staged in ("valu", "tm", "noq"):
            be.set_tuning("gram_q", 1)
        if staged in ("valu", "tm"):
            be.set_tuning("gram_tm", 1 if staged == "valu" else 2)
        if staged == "q":
            be.set_tuning("gram_q", 2)
    rng = np.random.default_rng(N + k)
    n = N * N
    Vh = np.linalg.qr(rng.standard_normal((n, k)))[0].T.copy()
    V = be.zeros(k, dev.slab.length)
    for j in range(k):
        V[j].copy_(dev.load(Vh[j]))
    u = 0.3 * rng.standard_normal(n)
    r = rng.standard_normal(n) * 1e3
    kp = be.gram_dim(k, with_r)
    W = np.zeros((n, kp))
    for j in range(k):
        W[:, j] = ref.jvp(u, Vh[j])
    if with_r:
        W[:, k] = r
    Rinv = None
    if with_rinv:
        A = np.triu(rng.standard_normal((kp, kp))) + 3 * np.eye(kp)
        A[k + (1 if with_r else 0):, :] = 0
        A[:, k + (1 if with_r else 0):] = 0
        if with_r:
            A[k, :] = 0
            A[:, k] = 0
            A[k, k] = 1.0
        Rinv = A
        W = W @ A
    Gref = W.T @ W
    Gd = be.zeros(kp * kp)
    be.gram(dev.load(u), V, k, None if Rinv is None else be.to_device(Rinv.reshape(-1)),
            dev.load(r) if with_r else None, Gd)
    Gdev = Gd.cpu().numpy().reshape(kp, kp)
    scale = np.sqrt(np.outer(np.diag(Gref), np.diag(Gref))) + 1e-300
    assert np.max(np.abs(Gdev - Gref) / scale) < 1e-13
    np.testing.assert_array_equal(Gdev, Gdev.T)


@pytest.mark.parametrize("staged", [0, 1])
def test_gram_deterministic(staged):
    prob, dev, ref = make(512)
    be = dev.backend
    be.set_tuning("gram_path", staged)
    rng = np.random.default_rng(3)
    k = 12
    V = be.zeros(k, dev.slab.length)
    for j in range(k):
        V[j].copy_(dev.load(rng.standard_normal(512 * 512)))
    u = dev.load(0.1 * rng.standard_normal(512 * 512))
    r = dev.load(rng.standard_normal(512 * 512))
    outs = []
    kp = be.gram_dim(k, True)
    rinv = be.to_device(np.eye(kp).reshape(-1) * 0.5)
    for _ in range(3):
        for ri in (None, rinv):
            Gd = be.zeros(kp ** 2)
            be.gram(u, V, k, ri, r, Gd)
            outs.append(Gd.cpu().numpy())
    for i in range(2, 6):
        np.testing.assert_array_equal(outs[i % 2], outs[i])


@pytest.mark.parametrize("N", [24, 100, 101, 512, 640, 1030])
def test_cg_matvec_matches_two_pass(N):
    """q = J^T J p (13-point fused) vs the oracle's two passes; even N runs the row-marching kernel,
    whose q must equal the point-wise kernel's bit for bit (same per-point arithmetic)."""
    prob, dev, ref = make(N)
    be = dev.backend
    rng = np.random.default_rng(N)
    n = N * N
    u = 0.3 * rng.standard_normal(n)
    p = rng.standard_normal(n)
    us, ps = dev.load(u), dev.load(p)
    d = dev.vec()
    be.jdiag(us, d)
    q = dev.vec()
    pq = dev.scalar(1)
    be.cg_matvec(d, ps, q, pq)
    q_ref = ref.vjp(u, ref.jvp(u, p))
    close(own(dev, q), q_ref, rtol=1e-12)
    np.testing.assert_allclose(pq.item(), p @ q_ref, rtol=1e-12)
    pq_again = dev.scalar(1)
    be.cg_matvec(d, ps, q, pq_again)
    assert pq_again.item() == pq.item()                            # deterministic reduction
    be.set_tuning("cg_matvec", 1)
    q0, pq0 = dev.vec(), dev.scalar(1)
    be.cg_matvec(d, ps, q0, pq0)
    np.testing.assert_array_equal(own(dev, q), own(dev, q0))
    np.testing.assert_allclose(pq0.item(), pq.item(), rtol=1e-13)


@pytest.mark.parametrize("N", [24, 100, 640])
@pytest.mark.parametrize("first", [True, False])
def test_cg_step_matvec_fused(N, first):
    """p_out = z + beta p_in (or z), x += alpha' p_in, q = J^T J p_out in one kernel: bit-identical to
    cg_update_p + cg_normal_matvec + the x update of cg_update_xr, ghost rows of p_out included."""
    prob, dev, ref = make(N)
    be = dev.backend
    rng = np.random.default_rng(N + first)
    n = N * N
    u = 0.3 * rng.standard_normal(n)
    us = dev.load(u)
    d = dev.vec()
    be.jdiag(us, d)
    z, p_in, x = (dev.load(rng.standard_normal(n)) for _ in range(3))
    beta, xalpha = 0.37, -1.3
    p_out, q, pq = dev.vec(), dev.vec(), dev.scalar(1)
    x_f = x.clone()
    be.cg_step_matvec(d, z, p_in, p_out, q, beta, first, None if first else x_f, xalpha, pq)
    # unfused reference sequence on the GPU
    p_ref = p_in.clone()
    be.cg_update_p(beta, first, z, p_ref)
    q_ref, pq_ref = dev.vec(), dev.scalar(1)
    be.cg_matvec(d, p_ref, q_ref, pq_ref)
    np.testing.assert_array_equal(p_out.cpu().numpy(), p_ref.cpu().numpy())    # whole slab (ghosts = 0)
    np.testing.assert_array_equal(own(dev, q), own(dev, q_ref))
    assert pq.item() == pq_ref.item()
    if not first:
        x_ref = x.clone()
        zero = dev.vec()
        be.cg_update_xr(xalpha, p_in, zero, x_ref, dev.vec(), None, dev.vec(), dev.scalar(2))
        np.testing.assert_array_equal(own(dev, x_f), own(dev, x_ref))


def test_cg_updates():
    prob, dev, ref = make(64)
    be = dev.backend
    rng = np.random.default_rng(5)
    n = 64 * 64
    p, q, x, r, dinv = (rng.standard_normal(n) for _ in range(5))
    ps, qs, xs, rs, ds = (dev.load(a) for a in (p, q, x, r, dinv))
    z = dev.vec()
    out = dev.scalar(2)
    be.cg_update_xr(0.7, ps, qs, xs, rs, ds, z, out)
    r2 = r - 0.7 * q
    np.testing.assert_array_equal(own(dev, xs), x + 0.7 * p)
    np.testing.assert_array_equal(own(dev, rs), r2)
    np.testing.assert_array_equal(own(dev, z), dinv * r2)
    np.testing.assert_allclose(out.cpu().numpy(), [r2 @ r2, r2 @ (dinv * r2)], rtol=1e-12)
    be.cg_update_p(0.3, False, z, ps)
    np.testing.assert_array_equal(own(dev, ps), p * 0.3 + dinv * r2)


def test_jvp_adjoint_and_linearity_8192():
    """Size-independent properties at the benchmark grid: <J v, w> = <v, J^T w>; J(a v) = a J v."""
    N = 8192
    prob, dev, ref = make(N)
    be = dev.backend
    g = torch.Generator(device=be.device).manual_seed(0)
    L = dev.slab.length

    def rnd():
        t = dev.vec()
        t[dev.slab.own] = torch.randn(N * N, generator=g, device=be.device, dtype=torch.float64)
        return t

    u, v, w = rnd(), rnd(), rnd()
    u.mul_(0.1)
    jv, jtw = dev.vec(), dev.vec()
    be.jvp(u, v, jv)
    be.vjp(u, w, jtw)
    a = torch.dot(jv[dev.slab.own], w[dev.slab.own]).item()
    b = torch.dot(v[dev.slab.own], jtw[dev.slab.own]).item()
    assert abs(a - b) <= 1e-11 * (abs(a) + torch.linalg.norm(jv).item() * torch.linalg.norm(w).item() * 1e-3)
    v2 = v * 2.0
    jv2 = dev.vec()
    be.jvp(u, v2, jv2)
    assert torch.equal(jv2, jv * 2.0)
    assert L == (N + 2 * G) * N


@pytest.mark.parametrize("k,rescale", [(1, True), (2, False), (7, True), (16, True), (21, True), (32, False)])
def test_lls_solve_device(k, rescale):
    """k_lls (one preconditioned CholeskyQR solve on the device) == the host algebra of lls.py
    (scipy Cholesky / triangular solves) to rounding: d, R, Ry, jdd to 1e-12 relative, e_try exact
    given the device d."""
    import scipy.linalg
    prob, dev, ref = make(24)
    be = dev.backend
    rng = np.random.default_rng(k)
    n = 400
    Y = rng.standard_normal((n, k + 1))
    Y[:, :k] = np.linalg.qr(Y[:, :k])[0] @ np.diag(rng.uniform(0.5, 2.0, k))
    if rescale:
        Y[:, k - 1] *= 1e3
    kp = be.gram_dim(k, True)
    Gh = np.zeros((kp, kp))
    Gh[:k + 1, :k + 1] = Y.T @ Y
    P = np.triu(rng.standard_normal((k, k))) + 3 * np.eye(k)
    if rescale:
        P[k - 1, :] = 0.0
        P[k - 1, k - 1] = 1.0
    sdd = rng.uniform(0.5, 2, k)
    e = rng.standard_normal(k)
    out = be.zeros(3 + k + 3 * k * k)
    etry = be.zeros(k)
    be.lls_solve(be.to_device(Gh.reshape(-1)), kp, k, be.to_device(P.reshape(-1)), rescale,
                 be.to_device(sdd), be.to_device(e), out, etry)
    o = out.cpu().numpy()
    g = Gh[:k + 1, :k + 1].copy()
    p = P.copy()
    if rescale:
        s = np.sqrt(g[k - 1, k - 1])
        g[k - 1, :] /= s
        g[:, k - 1] /= s
        p[k - 1, k - 1] = s
        assert o[2] == s
    ry = scipy.linalg.cholesky(g[:k, :k], lower=False)
    z = scipy.linalg.solve_triangular(ry, g[:k, k], trans="T", lower=False)
    R = ry @ p
    d = -scipy.linalg.solve_triangular(R, z, lower=False)
    assert o[0] == 0.0
    np.testing.assert_allclose(o[3:3 + k], d, rtol=1e-11, atol=1e-12 * np.abs(d).max())
    np.testing.assert_allclose(o[3 + k:3 + k + k * k].reshape(k, k), R, rtol=1e-12, atol=1e-13 * np.abs(R).max())
    np.testing.assert_allclose(o[3 + k + k * k:3 + k + 2 * k * k].reshape(k, k), ry, rtol=1e-12, atol=1e-13 * np.abs(ry).max())
    np.testing.assert_allclose(o[1], np.sum((R @ d) ** 2), rtol=1e-11)
    np.testing.assert_array_equal(etry.cpu().numpy(), e + sdd * o[3:3 + k])
    np.testing.assert_allclose(o[3 + k + 2 * k * k:].reshape(k, k) @ R, np.eye(k), rtol=0, atol=1e-12)
    # not SPD -> status 1
    Gb = Gh.copy()
    Gb[0, 0] = -1.0
    be.lls_solve(be.to_device(Gb.reshape(-1)), kp, k, be.to_device(P.reshape(-1)), False,
                 be.to_device(sdd), be.to_device(e), out, etry)
    assert out[0].item() == 1.0


@pytest.mark.parametrize("k,pending", [(1, False), (1, True), (5, True), (12, False), (20, True), (31, True)])
def test_lls_next_device(k, pending):
    """k_lls_next (the next step's transform / preconditioner / scales) == the NumPy
    double of the same bookkeeping (tests/numpy_backend.py), and k_lls's R^-1 block == R^-1."""
    from tests.numpy_backend import NumpyBackend
    prob, dev, ref = make(24)
    be = dev.backend
    rng = np.random.default_rng(100 + k)
    kp = be.gram_dim(k, True)
    Y = rng.standard_normal((300, k + 1))
    Gh = np.zeros((kp, kp))
    Gh[:k + 1, :k + 1] = Y.T @ Y
    P = np.triu(rng.standard_normal((k, k))) + 3 * np.eye(k)
    sdd, e = rng.uniform(0.5, 2, k), rng.standard_normal(k)
    out, etry = be.zeros(3 + k + 3 * k * k), be.zeros(k)
    be.lls_solve(be.to_device(Gh.reshape(-1)), kp, k, be.to_device(P.reshape(-1)), True, be.to_device(sdd),
                 be.to_device(e), out, etry)
    o = out.cpu().numpy()
    R = o[3 + k:3 + k + k * k].reshape(k, k)
    Rinv = o[3 + k + 2 * k * k:].reshape(k, k)
    np.testing.assert_allclose(Rinv @ R, np.eye(k), rtol=0, atol=1e-12)
    pack = np.concatenate([[1.0, rng.uniform(0.5, 3.0), 0.1], rng.standard_normal(k)])
    sc = rng.uniform(0.5, 2.0, k)
    kpn = be.gram_dim(k + 1, True)
    nb = NumpyBackend()
    dv = [be.zeros(n) for n in (kpn * kpn, (k + 1) ** 2, k + 1, k + 1, k, k)]
    hv = [torch.zeros(n, dtype=torch.float64) for n in (kpn * kpn, (k + 1) ** 2, k + 1, k + 1, k, k)]
    be.lls_next(k, pending, out, etry, be.to_device(pack), be.to_device(sc), kpn, *dv)
    nb.lls_next(k, pending, out.cpu(), etry.cpu(), torch.from_numpy(pack), torch.from_numpy(sc), kpn, *hv)
    for d_, h_ in zip(dv, hv):
        np.testing.assert_allclose(d_.cpu().numpy(), h_.numpy(), rtol=1e-15, atol=0)


@pytest.mark.parametrize("world,n", [(1, 5), (2, 1), (3, 441), (8, 3000), (6, 70), (13, 33)])
def test_rank_sum_matches_host_order(world, n):
    """gnk_rank_sum == the host's sum over ranks (slab.tree_sum, slab.Comm), bit for bit."""
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import tree_sum
    prob, dev, ref = make(24)
    be = dev.backend
    parts = np.random.default_rng(world * n).standard_normal((world, n)) * 10.0 ** np.arange(world)[:, None]
    out = be.zeros(n)
    be.rank_sum(be.to_device(parts.reshape(-1)), world, out)
    np.testing.assert_array_equal(out.cpu().numpy(), tree_sum(parts))


def test_timer_classes_and_stream_probe():
    """The bench's per-launch timer with two classes in one window (Gram + first trial), launch order
    and class ids kept; the streaming-floor probe computes triad / copy / read exactly."""
    prob, dev, ref = make(1024)
    be = dev.backend
    n = 1 << 20
    a = be.zeros(n)
    b = torch.arange(n, dtype=torch.float64, device=a.device)
    c = torch.full((n,), 3.0, dtype=torch.float64, device=a.device)
    be.timer_start(_native.TIMER_PROBE, 8)
    be.timer_add(_native.TIMER_JVP)
    be.probe_stream(a, b, c, 0.5, n, 0)
    torch.testing.assert_close(a, b + 1.5, rtol=0, atol=0)
    be.probe_stream(a, c, None, 0.0, n, 2)
    torch.testing.assert_close(a, c, rtol=0, atol=0)
    be.probe_stream(None, b, None, 0.0, n, 1)
    u = dev.load(np.zeros(1024 * 1024))
    be.jvp(u, u, dev.vec())
    got = be.timer_collect_ids(8)
    assert [i for i, _, _ in got] == [_native.TIMER_PROBE] * 3 + [_native.TIMER_JVP]
    assert [by for _, _, by in got] == [24.0 * n, 16.0 * n, 8.0 * n, 24.0 * 1024 * 1024]
    assert all(ms > 0 for _, ms, _ in got)
