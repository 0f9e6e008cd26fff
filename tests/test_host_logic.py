"""Host-side logic of the device solvers, on CPU.

The GNK / GN drivers, the CholQR2 least-squares solve and the slab bookkeeping
run here against the NumPy test double of the C-ABI (tests/numpy_backend.py) and
are checked against the reference's golden fixtures.  The HIP kernels
themselves are covered by the -m gpu tests.
"""
import contextlib
import io

import numpy as np
import pytest

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
from oracle import gnk_oracle as O
from tests.numpy_backend import NumpyBackend

RTOL = 1e-10


def run(method, prob_kw, u0, y, **kw):
    prob = gnk.BratuPdeProblem(**prob_kw)
    ref_prob = O.BratuPdeProblem(**prob_kw)
    ref_res = ref_prob.make_res(y)
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
            out = method(prob.make_res(y), u0, prob.make_jac(), callback=cb, _backend=NumpyBackend(), **kw)
        except gnk.StepLengthConvergenceError as e:
            exc = ["StepLengthConvergenceError", e.message]
    return out, rec, buf.getvalue().splitlines(), exc


def check(case, out, rec, so, exc, rtol=RTOL, fragile_last=False):
    """fragile_last: the converged final step's Armijo test is a rounding tie
    (prev - cur ~ 0.5 t ||J d||^2 ~ ulp(||r||^2)), so only that step's
    trial count (and hence nrev) may differ."""
    assert so == case["stdout"]
    assert (exc is None) == (case["exception"] is None)
    if out is not None:
        assert (out.nit, out.njev, out.success) == (case["nit"], case["njev"], case["success"])
        if not fragile_last:
            assert out.nrev == case["nrev"]
    ref = case["per_iter"]
    if fragile_last:
        assert rec["nfev"][:-1] == ref["nfev"][:-1]
    else:
        assert rec["nfev"] == ref["nfev"]
    assert rec["cg_iter"] == ref["cg_iter"]
    np.testing.assert_allclose(rec["xnorm"], ref["xnorm"], rtol=rtol)
    np.testing.assert_allclose(rec["rnorm"], ref["rnorm"], rtol=rtol, atol=RTOL * ref["rnorm"][0])


@pytest.mark.parametrize("version", ["res_old", "res_new", "jac_old_res_old", "jac_old_res_new"])
def test_gnk_bratu24_no_restart(golden, version):
    meta, arr = golden
    out, rec, so, exc = run(gnk.gauss_newton_krylow, dict(grid_nodes=25, ALPHA=5, LAMBDA=10),
                            arr["bratu24_u0"], arr["bratu24_y"], version=version, max_iter=100)
    check(meta["cases"][f"bratu24_{version}_rNone"], out, rec, so, exc)
    np.testing.assert_allclose(out.x, meta and arr[f"bratu24_{version}_rNone__x"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("version", ["res_old", "res_new"])
def test_gnk_bratu24_restart20(golden, version):
    meta, arr = golden
    out, rec, so, exc = run(gnk.gauss_newton_krylow, dict(grid_nodes=25, ALPHA=5, LAMBDA=10),
                            arr["bratu24_u0"], arr["bratu24_y"], version=version, max_iter=100, krylow_restart=20)
    check(meta["cases"][f"bratu24_{version}_r20"], out, rec, so, exc, rtol=1e-10, fragile_last=True)


def test_gnk_bratu24_linear_breakdown(golden):
    meta, arr = golden
    prob = O.BratuPdeProblem(25, 5, 0.0)
    y = prob.pde_operator(prob.u_true)
    out, rec, so, exc = run(gnk.gauss_newton_krylow, dict(grid_nodes=25, ALPHA=5, LAMBDA=0.0),
                            arr["bratu24_linear_u0"], y, max_iter=100)
    assert so == meta["cases"]["bratu24_linear_res_old"]["stdout"]
    assert exc is not None


def test_gn_bratu24(golden):
    meta, arr = golden
    for name, kw in (("bratu24_gn", {}), ("bratu24_gn_precond", {"cg_preconditioner": True})):
        out, rec, so, exc = run(gnk.gauss_newton, dict(grid_nodes=25, ALPHA=5, LAMBDA=10),
                                arr["bratu24_u0"], arr["bratu24_y"], **kw)
        check(meta["cases"][name], out, rec, so, exc, rtol=1e-9)


def test_row_partition_covers_grid():
    for N in (5, 24, 100, 8192):
        for P in (1, 2, 3, 8):
            parts = [gnk.row_partition(N, P, p) for p in range(P)]
            assert parts[0][0] == 0
            assert sum(n for _, n in parts) == N
            for (a0, an), (b0, _) in zip(parts, parts[1:]):
                assert a0 + an == b0


@pytest.mark.parametrize("name,kw", [("bratu24_gn", {}), ("bratu24_gn_precond", {"cg_preconditioner": True})])
def test_gn_single_reduction_cg(golden, name, kw):
    """cg_variant="single_reduction" (Chronopoulos-Gear): not bit-compatible with scipy's
    recurrence, but on the golden GN runs the CG counts and the outer bookkeeping are unchanged and
    the iterates agree to 1e-9."""
    meta, arr = golden
    out, rec, so, exc = run(gnk.gauss_newton, dict(grid_nodes=25, ALPHA=5, LAMBDA=10), arr["bratu24_u0"],
                            arr["bratu24_y"], cg_variant="single_reduction", **kw)
    check(meta["cases"][name], out, rec, so, exc, rtol=1e-9)


@pytest.mark.parametrize("restart,version", [(3, "res_old"), (5, "res_new")])
def test_gnk_short_restart_cycles_vs_oracle(restart, version):
    """N = 256, short restart cycles: the speculative next-step solve across many restarts (DESIGN.md
    §5b) keeps the oracle's bookkeeping; ||x_k|| within 5e-9 (post-restart LS steps are
    cancellation-limited)."""
    N = 256
    prob_o, y, u0 = O.bratu_workload(N)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    rd, ro = [], []
    with contextlib.redirect_stdout(io.StringIO()):
        out = gnk.gauss_newton_krylow(prob.make_res(y), u0, prob.make_jac(), krylow_restart=restart, max_iter=40,
                                      version=version, _backend=NumpyBackend(),
                                      callback=lambda x, nfev, cg_iter: rd.append((np.linalg.norm(x), nfev)))
        ref = O.gauss_newton_krylow(prob_o.make_res(y), u0, prob_o.make_jac(), krylow_restart=restart, max_iter=40,
                                    version=version,
                                    callback=lambda x, nfev, cg_iter: ro.append((np.linalg.norm(x), nfev)))
    assert (out.nit, out.nrev, out.njev, out.success) == (ref.nit, ref.nrev, ref.njev, ref.success)
    assert [n for _, n in rd] == [n for _, n in ro]
    np.testing.assert_allclose([a for a, _ in rd], [a for a, _ in ro], rtol=5e-9)


class _FakeDev:
    """The pieces of a BratuDevice that lls.CholQR2Solver reads, around the NumPy test double."""

    def __init__(self, n):
        from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
        self.backend = NumpyBackend()
        self.comm = Comm(single=True)
        self.slab = type("S", (), {"n_global": n})()


class _PendingBasis:
    k = 1
    pending = True
    V = None
    sc = np.ones(4)

    def gram_k(self):
        return 2

    def gram_left(self):
        return None


def test_pending_singular_solve_drops_preconditioner():
    """A solve over a pending column whose Gram stays numerically singular (every pass needs the shift)
    takes the minimum-norm branch; once the pending column settles, that rank-deficient R must not
    become the next pass's preconditioner (resolve_pending kept it)."""
    from gauss_newton_via_generalized_krylov_subspaces_amd.lls import CholQR2Solver
    n = 1000
    dev = _FakeDev(n)
    G0 = np.diag([1.0, -1e-30, 1.0])           # [J V | r] Gram with an indefinite (singular) k x k block
    G0[0, 2] = G0[2, 0] = 0.5

    def gram(u, V, k, rinv, r, G):
        kp = dev.backend.gram_dim(k, r is not None)
        g = np.zeros((kp, kp))
        m = min(kp, 3) if r is not None else min(kp, 2)
        g[:m, :m] = G0[:m, :m]
        G.numpy()[:kp * kp] = g.reshape(-1)

    ls = CholQR2Solver(dev, 4, gram=gram, n_global=n, device_solve=False)
    ls.R_prev = np.eye(1)                        # a usable factor of the settled column
    with contextlib.redirect_stdout(io.StringIO()) as out:
        d, jdd, R = ls.solve(None, _PendingBasis(), None)
        assert np.all(np.isfinite(d))
        d2 = ls.resolve_pending(2.0)
    assert ls.R_prev is None and np.all(np.isfinite(d2))
    assert "A is rank deficient" in out.getvalue()
    assert ls._initial_preconditioner(3) == (None, False)      # next solve: CholQR2 from scratch


def test_generic_wide_gram_arena_guard():
    """A generic basis wider than 63 columns whose Y = W RinvAug exceeds the library's scratch arena is
    refused with NotImplementedError up front, not by a native error mid-run."""
    from gauss_newton_via_generalized_krylov_subspaces_amd.generic import HostCallableOps

    class SmallArena(NumpyBackend):
        def scratch_doubles(self):
            return 80 * 1000

    ops = HostCallableOps(lambda x: x, lambda x: np.eye(x.size), 4, backend=SmallArena())
    ops.m = 2000
    with pytest.raises(NotImplementedError, match="krylow_restart <= 63") as ei:
        ops.gram(None, None, 70, None, ops.be.zeros(2000), ops.be.zeros(96 * 96))
    # the suggested bound is the real limit: kp = gram_dim(k, r) rounds k + 1 up to 16, and
    # kp <= 64 needs no arena
    kb = int(str(ei.value).rsplit("<= ", 1)[1].rstrip(")"))
    assert ops.be.gram_dim(kb, True) <= 64
    assert ops.be.gram_dim(kb + 1, True) * ops.m > ops.be.scratch_doubles()
    ops.m = 500                                       # arena 80 000 / 500 -> kp 160: k <= 159
    assert ops.max_arena_k(True) == 159
    assert ops.be.gram_dim(159, True) * ops.m <= ops.be.scratch_doubles() < ops.be.gram_dim(160, True) * ops.m


def test_tree_sum_is_the_subtree_fold_of_every_power_of_two_partition():
    """slab.tree_sum (= gnk_rank_sum's and gnk_set_segments' fold order): folding 8 segments on one rank
    equals folding each rank's 8 / w segments and then the w rank values, bit for bit, for w | 8 -- the
    property that makes segment reductions rank-count independent.  Also the device's binary-counter form
    of the same order (k_rank_sum) for every count up to 40."""
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import reduction_segments, tree_sum
    rng = np.random.default_rng(5)
    for _ in range(200):
        seg = rng.standard_normal((8, 7)) * 10.0 ** rng.integers(-8, 8, size=(8, 7))
        one = tree_sum(seg)
        for w in (2, 4, 8):
            ranks = np.stack([tree_sum(seg[p * (8 // w):(p + 1) * (8 // w)]) for p in range(w)])
            assert np.array_equal(tree_sum(ranks), one)

    def counter_fold(vals):                      # k_rank_sum's stack form
        sv, sz = [], []
        for v in vals:
            z = 1
            while sz and sz[-1] == z:
                v = sv.pop() + v
                sz.pop()
                z *= 2
            sv.append(v)
            sz.append(z)
        s = sv.pop()
        while sv:
            s = sv.pop() + s
        return s
    for n in range(1, 41):
        vals = rng.standard_normal(n) * 10.0 ** rng.integers(-10, 10, size=n)
        assert counter_fold(list(vals)) == tree_sum(vals[:, None])[0]
    assert reduction_segments(8192, 8, None) == 1024 and reduction_segments(8192, 1, None) == 0
    assert reduction_segments(8192, 1, True) == 1024 and reduction_segments(8192, 4, False) == 0
    assert reduction_segments(384, 3, None) == 0 and reduction_segments(100, 2, None) == 0


def _cg_paths(backend_factory, N=64, maxiter=None, rtol=1e-8, pre=True):
    """The fused CGLS solve three ways on one Bratu slab: host scalars (``_cg_fused``), device scalars
    with the lagged stopping read, and device scalars read every iteration -> {name: (x, iterations)}."""
    from gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton import BratuGNOps, DeviceCG
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
    ref_prob, y, u0 = O.bratu_workload(N)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    out = {}
    for name, dev, lag in (("host", False, False), ("device_lagged", True, True), ("device", True, False)):
        ops = BratuGNOps(prob, y, Comm(single=True), backend=backend_factory())
        u = ops.load(u0)
        r0 = ops.vec()
        ops.residual(u, r0)
        cg = DeviceCG(ops)
        cg.device_scalars, cg.lag_reads = dev, lag
        x, it = cg.solve(u, r0, cg_rtol=rtol, preconditioner=pre, maxiter=maxiter)
        out[name] = (x[ops.dev.slab.own].cpu().numpy().copy(), it)
    return out


@pytest.mark.parametrize("maxiter,pre", [(None, True), (None, False), (7, True), (0, True), (0, False)])
def test_cg_device_scalars_bit_identical(maxiter, pre):
    """the fused CG with its scalar recurrence on the device (gnk_cg_scalars, lagged read)
    gives the host-scalar path's iterates and counts bit for bit -- to convergence and at the cap (maxiter 0:
    scipy runs no iteration, x = 0)."""
    got = _cg_paths(NumpyBackend, maxiter=maxiter, pre=pre)
    xh, ih = got["host"]
    if maxiter == 0:
        assert ih == 0 and not np.any(xh)
    else:
        assert ih > 5
    for name in ("device_lagged", "device"):
        x, it = got[name]
        assert it == ih and np.array_equal(x, xh), name
