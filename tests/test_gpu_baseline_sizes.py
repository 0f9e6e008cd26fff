"""Parity at BASELINE.json's sizes against the REFERENCE's own outputs (tests/golden/large_*.json,
written by tests/golden/make_golden_large.py, which ran the reference in the build container).

* C2 (configs[1]): Bratu N = 1024, krylow_restart = 20, max_iter = 100 -- the whole run, res_old
  and res_new (ref:gauss_newton_krylow.py:84-136).
* Headline bench workload: N = 8192, restart 20, res_old, the first 4 outer iterations (k = 1..4).
* C3 (configs[2]): N = 8192, the first Gauss-Newton step's CGLS (Jacobi, rtol 1e-8,
  ref:gauss_newton.py:50-58) capped at 30 CG iterations.

Tolerances (per-iteration ||x_k|| and ||r_k||, relative): max(1e-10, envelope_i), envelope_i = the
largest move of the reference's own trajectory at iteration i under algebraically equivalent
reorderings of its arithmetic (tests/tolerances.py, tests/golden/sensitivity.json).  At these sizes
the envelope is large in two places: iteration 1 (k = 1), where ||x_1|| = |c + d| cancels to 1e-5 of
||x_0|| and the reference's own dot products are 4e-10 (N = 1024) / 6e-8 (N = 8192) away from the
exactly rounded step, and res_old after its first restart (iteration > 21), whose trajectory is
chaotic (1e-7 under a row permutation of the QR).  The converged last step of the res_old run is an
Armijo rounding tie (its trial count moves with the reorderings too).
"""
import contextlib
import io
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from oracle import gnk_oracle as O  # noqa: E402
from tests import tolerances as T  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL = T.NORTH_STAR


def _load(name):
    with open(os.path.join(GOLDEN, f"large_{name}.json")) as f:
        meta = json.load(f)
    arr = dict(np.load(os.path.join(GOLDEN, f"large_{name}.npz")))
    return meta, arr


def _run_gnk(N, max_iter, version):
    prob_o, y, u0 = O.bratu_workload(N)
    res_o = prob_o.make_res(y)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    rec = {"xnorm": [], "rnorm": [], "nfev": []}

    def cb(x, nfev, cg_iter):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(res_o(x))))
        rec["nfev"].append(nfev)

    buf = io.StringIO()
    # gauss_newton_krylow's own steps (the same GNKSolver it builds for make_res / make_jac), kept so the
    # test can read the per-step Armijo comparisons of the trace
    s = gnk.GNKSolver(prob, y, krylow_restart=20, max_iter=max_iter, version=version, callback=cb)
    with contextlib.redirect_stdout(buf):
        s.setup(u0)
        while not s.step():
            pass
        out = s.finish()
    rec["trace"] = s.trace
    return out, rec, buf.getvalue().splitlines()


@pytest.mark.parametrize("version", ["res_old", "res_new"])
def test_c2_full_run_vs_reference(version):
    meta, arr = _load("c2")
    case = meta["cases"][version]
    out, rec, so = _run_gnk(1024, 100, version)
    ref = case["per_iter"]
    n = len(ref["nfev"])
    assert so == case["stdout"]
    assert (out.nit, out.njev, out.success) == (case["nit"], case["njev"], case["success"])
    assert len(rec["nfev"]) == n
    last_tie = version == "res_old" and case["success"]
    m = n - 1 if last_tie else n
    assert rec["nfev"][:m] == ref["nfev"][:m]
    if last_tie:                   # the converged step's Armijo count is a rounding tie
        seen = T.last_nfev_values(f"c2_{version}")
        print(f"C2 {version}: last step nfev {rec['nfev'][-1]} (reference {ref['nfev'][-1]}, the counts of its "
              f"reorderings {seen})")
        # the device's count is one the reference's own arithmetic, reordered, produces (tests/tolerances.py)
        assert rec["nfev"][-1] in seen and out.nrev - rec["nfev"][-1] == case["nrev"] - ref["nfev"][-1]
        # ... and it is the device's own tracked count: drift inside the family's range is seen too
        assert rec["nfev"][-1] == T.DEVICE_LAST_NFEV[f"c2_{version}"], rec["nfev"][-1]
        # ... and why it is a tie: the step's Armijo threshold 0.5 t ||J d||^2 (t <= 1) is below one ulp of the
        # loss, so every trial's decision (ref:armijo_goldstein.py:57-62) is the sign of the rounding noise of
        # sum r^2 -- which stays within a few ulps of the previous loss at every trial point
        last = rec["trace"][-1]
        ulp = np.finfo(np.float64).eps * last["prev_loss"]
        noise = [(last["prev_loss"] - c) / ulp for c in last["losses"]]
        print(f"C2 {version}: last step 0.5 ||J d||^2 = {0.5 * last['jdd'] / ulp:.3g} ulp of the loss; "
              f"prev - cur per trial, in ulps: {np.round(noise, 2).tolist()}")
        assert 0.5 * last["jdd"] < ulp and len(noise) == rec["nfev"][-1] - rec["nfev"][-2]
        assert max(abs(v) for v in noise) <= T.ARMIJO_TIE_ULPS, noise
    else:
        assert out.nrev == case["nrev"]
    tol = T.per_iteration(f"c2_{version}", n)
    tol_r = T.per_iteration(f"c2_{version}", n, "r")
    ex = np.abs(np.array(rec["xnorm"]) - ref["xnorm"]) / np.abs(ref["xnorm"])
    er = np.abs(np.array(rec["rnorm"]) - ref["rnorm"]) / np.abs(ref["rnorm"])
    print(f"C2 {version}: max rel ||x_k|| {ex.max():.3g} (it {ex.argmax() + 1}), k=1 {ex[0]:.3g}, "
          f"before restart {ex[1:21].max():.3g}; ||r_k|| {er.max():.3g}")
    assert np.all(ex <= tol), np.nonzero(ex > tol)
    assert np.all(er <= tol_r), np.nonzero(er > tol_r)
    xs = out.x[::meta["subsample_stride"]]
    np.testing.assert_allclose(xs, arr[f"{version}__x_sub"], rtol=0, atol=tol[-1] * 10 * np.abs(xs).max())


def test_headline_8192_first_iterations_vs_reference():
    """The bench workload (8192^2, restart 20, res_old): the first 4 outer iterations (k = 1..4)."""
    meta, _ = _load("head8192")
    case = meta["cases"]["res_old"]
    out, rec, so = _run_gnk(8192, 5, "res_old")
    ref = case["per_iter"]
    assert (out.nit, out.nrev, out.njev, out.success) == (case["nit"], case["nrev"], case["njev"], case["success"])
    assert rec["nfev"] == ref["nfev"] and so == case["stdout"]
    tol = T.per_iteration("head8192", len(ref["nfev"]))
    tol_r = T.per_iteration("head8192", len(ref["nfev"]), "r")
    ex = np.abs(np.array(rec["xnorm"]) - ref["xnorm"]) / np.abs(ref["xnorm"])
    er = np.abs(np.array(rec["rnorm"]) - ref["rnorm"]) / np.abs(ref["rnorm"])
    print(f"8192^2 first 4 iterations: rel ||x_k|| {ex}, ||r_k|| {er}")
    assert np.all(ex <= tol) and np.all(er <= tol_r)


def test_c3_cgls_8192_capped_vs_reference():
    """C3: CGLS of the first GN step at 8192^2 (A = -J(u0), y = res(u0), Jacobi, rtol 1e-8), 30
    iterations of the scipy recurrence on the device vs scipy.sparse.linalg.cg on the reference's
    CSR operator: per-iteration ||x_k||, the final true normal-equation residual, x subsampled."""
    from gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton import BratuGNOps, DeviceCG
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
    meta, arr = _load("c3")
    N = 8192
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    dev = BratuDevice(prob, Comm(single=True))
    u0, y, _ = slab_inputs(dev)
    ops = BratuGNOps(prob, y, Comm(single=True), backend=dev.backend)
    u = ops.load(u0)
    r0 = ops.vec()
    ops.residual(u, r0)
    cg = DeviceCG(ops)
    own = dev.slab.own
    seen = []
    x, iters = cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=meta["cg_cap"],
                        callback=lambda xk: seen.append(float(torch.linalg.norm(xk[own]))))
    assert iters == meta["cg_cap"] == meta["info"]
    xnorm = seen[1:] + [float(torch.linalg.norm(x[own]))] if cg.p2 is not None else seen
    ref = np.array(meta["per_iter"]["xnorm"])
    ex = np.abs(np.array(xnorm) - ref) / ref
    xh = x[own].cpu().numpy()
    # the true normal-equation residual at the final iterate, on the host (oracle stencils)
    prob_o, y_o, u0_o = O.bratu_workload(N)
    J = prob_o.make_jac()(u0_o)
    b = -(J.T @ prob_o.make_res(y_o)(u0_o))
    rn = float(np.linalg.norm(b - (J.T @ (J @ xh))))
    print(f"C3 CGLS 8192^2: max rel ||x_k|| {ex.max():.3g}; final ||A^T y - A^T A x|| rel "
          f"{abs(rn - meta['per_iter']['resnorm'][-1]) / meta['per_iter']['resnorm'][-1]:.3g}")
    assert np.all(ex <= TOL)
    np.testing.assert_allclose(rn, meta["per_iter"]["resnorm"][-1], rtol=1e-8)
    xs = xh[::meta["subsample_stride"]]
    np.testing.assert_allclose(xs, arr["x_sub"], rtol=0, atol=TOL * np.abs(xs).max())


def test_headline_8192_full_restart_cycle_vs_oracle():
    """The bench workload over one whole restart cycle (8192^2, restart 20, res_old: iterations 1..20 at
    k = 1..20, then the restart and iteration 21 at k = 1) against the pinned oracle run in the build
    container (tests/golden/make_cycle8192.py: the reference does not fit there at k = 20; its lean
    restatement reproduces the reference's own head8192 fixture to 5e-13).  This pins the staged MFMA
    Gram passes that dominate the timed window (k = 10..20, ref:gauss_newton_krylow.py:86-89) on the
    real trajectory.  Bookkeeping (per-iteration nfev, basis size) exact.  Three oracle variants, all
    evaluations of the reference algorithm that differ only in rounding / factorisation:
      * base -- the reference's arithmetic (numpy dots, LAPACK Householder QR);
      * exact_k1 -- base with its cancellation-limited k = 1 sums exactly rounded (math.fsum);
      * cholqr -- the device's least-squares arithmetic (k_lls's k = 1 step on exact sums, preconditioned
        CholeskyQR on an extended-precision Gram) on the reference's own basis.
    E_i = |exact_k1_i - base_i| is how far the reference's own trajectory moves when only its k = 1 sums
    are re-rounded (1e-7 at iterations 3-4: ||x_1|| cancels ||x_0|| to 1e-8, u ||x_0|| / ||x_1|| ~ 1e-8).
    Asserted, per iteration, for ||x_k|| and ||r_k||: the device is within max(1e-10, E_i) of exact_k1
    (measured ~10x inside: the device's k = 1 step is closer to the exactly rounded one than the
    reference's), hence within 2 E_i of base by the triangle inequality (round 3's bound, now derived
    instead of assumed); within max(1e-10, E_i / 3) of cholqr, and at iteration 1 (k = 1) equal to it to
    1e-14.  |cholqr - exact_k1| (the factorisation's own move) is printed."""
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
    with open(os.path.join(GOLDEN, "large_cycle8192.json")) as f:
        fx = json.load(f)
    base, ex, ch = fx["variants"]["base"], fx["variants"]["exact_k1"], fx["variants"]["cholqr"]
    N = fx["N"]
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    comm = Comm(single=True)
    dev = BratuDevice(prob, comm)
    u0, y, _ = slab_inputs(dev)
    own = dev.slab.own
    xs, rs, nf = [], [], []

    def cb(x, nfev, cg_iter):
        xs.append(float(torch.linalg.norm(x.x[own])))
        rs.append(float(np.sqrt(x.sumsq)))
        nf.append(int(nfev))

    s = gnk.GNKSolver(prob, y, comm=comm, backend=dev.backend, callback=cb, callback_format="device",
                      **fx["kwargs"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        s.setup(u0)
        while not s.step():
            pass
    ks = [t["k"] for t in s.trace]
    assert ks == base["k"] == ch["k"] and nf == base["nfev"] == ch["nfev"], (ks, nf)
    assert buf.getvalue().splitlines() == base["stdout"]          # rank / breakdown messages (none expected)
    n = len(base["xnorm"])

    def rel(a, b):
        return np.abs(np.array(a[:n]) - np.array(b[:n])) / np.abs(np.array(b[:n]))

    E_x = np.maximum(TOL, rel(ex["xnorm"], base["xnorm"]))
    E_r = np.maximum(TOL, rel(ex["rnorm"], base["rnorm"]))
    p2 = lambda a: np.array2string(a, precision=2)                # noqa: E731
    dxe, dre = rel(xs, ex["xnorm"]), rel(rs, ex["rnorm"])
    dxc, drc = rel(xs, ch["xnorm"]), rel(rs, ch["rnorm"])
    print(f"8192^2 cycle ({n} iterations), relative per iteration:")
    print(f"  ||x_k|| device vs exact_k1 {p2(dxe)}")
    print(f"  ||x_k|| device vs cholqr   {p2(dxc)}")
    print(f"  ||x_k|| device vs base     {p2(rel(xs, base['xnorm']))}")
    print(f"  bound E_i = max(1e-10, |exact_k1 - base|) {p2(E_x)}")
    print(f"  |cholqr - exact_k1| {p2(rel(ch['xnorm'], ex['xnorm']))}")
    print(f"  ||r_k|| device vs exact_k1 {p2(dre)}; vs cholqr {p2(drc)}; bound {p2(E_r)}")
    print(f"  device least-squares passes per solve {s.lls.passes / max(1, len(s.lls.history)):.3f}; "
          f"oracle cholqr passes {[p[1] for p in ch['ls_passes']]}")
    assert np.all(dxe <= E_x) and np.all(dre <= E_r), (np.nonzero(dxe > E_x), np.nonzero(dre > E_r))
    # the cholqr variant runs the device's least-squares arithmetic: the kernels add less than a third of
    # what one re-rounding of the reference's k = 1 sums moves its own trajectory (measured 40x less for
    # ||x_k||, 4x for ||r_k||), and the k = 1 step itself is the same step (measured 1.3e-16: the device's
    # k = 1 Gram sums round like exactly rounded ones)
    bx, br = np.maximum(TOL, E_x / 3), np.maximum(TOL, E_r / 3)
    assert np.all(dxc <= bx) and np.all(drc <= br), (np.nonzero(dxc > bx), np.nonzero(drc > br))
    assert dxc[0] <= 1e-14 and dxc[n - 1] <= 1e-9, (dxc[0], dxc[n - 1])
