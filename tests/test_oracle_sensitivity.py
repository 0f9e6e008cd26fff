"""Documents which golden trajectories are chaotic in the REFERENCE algorithm itself.

The linear Bratu run with version='res_new' (ref:bratu_pde_test.py:277-318 at grid 25)
grows the basis to 177 columns; near breakdown the projected normal residual is
mostly rounding noise, so its normalisation (ref:krylow.py:71) amplifies any
perturbation.  Here a 1e-13 relative perturbation of each least-squares step of the
oracle (which matches the reference to 1e-10 unperturbed) changes ||x_k|| by >1e-6
in the middle of the run although cond(J V) <= 65 throughout -- so no
implementation with a different rounding can be held to 1e-10 there.
"""
import contextlib
import io

import numpy as np

from oracle import gnk_oracle as O


def test_linear_res_new_trajectory_is_chaotic():
    prob, y, u0 = O.bratu_workload(24, lam=0.0, linear_u0=True)
    res, jac = prob.make_res(y), prob.make_jac()
    orig = O.linear_least_squares
    runs = []
    for pert in (0.0, 1e-13):
        xs = []
        O.linear_least_squares = (lambda A, yy, p=pert: orig(A, yy) * (1 + p))
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                O.gauss_newton_krylow(res, u0, jac, version="res_new", max_iter=200,
                                      callback=lambda x, nfev, cg_iter: xs.append(np.linalg.norm(x)))
        finally:
            O.linear_least_squares = orig
        runs.append(np.array(xs))
    rel = np.abs(runs[0] - runs[1]) / np.abs(runs[0])
    assert rel[1:30].max() < 1e-12         # insensitive early (step 0 is cancellation-limited)
    assert rel.max() > 1e-6                # amplified by ~1e7 in the near-breakdown phase
    assert rel[-1] < 1e-10                 # re-converges to the same solution


# ---------------------------------------------------------------------------------------------------
# Evidence for the GPU parity bounds (tests/tolerances.py).  Each test recomputes, on the oracle, how far
# an algebraically equivalent reordering of the reference's own arithmetic moves the reference result.
import json  # noqa: E402
import math  # noqa: E402
import os  # noqa: E402
import sys  # noqa: E402

import pytest  # noqa: E402

from tests import tolerances as T  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import make_sensitivity as MS  # noqa: E402


def _fdot(a, b):
    return math.fsum(a * b)


def scipy_cg_exact(matvec, b, psolve=None, rtol=1e-5, maxiter=None, callback=None):
    """O.scipy_cg (scipy 1.15.3 cg) with every dot product / norm an exactly rounded sum."""
    bnrm2 = math.sqrt(_fdot(b, b))
    atol = max(0.0, float(rtol) * bnrm2)
    if bnrm2 == 0:
        return b, 0
    maxiter = len(b) * 10 if maxiter is None else maxiter
    x, r, rho_prev, p = np.zeros_like(b), b.copy(), None, None
    for it in range(maxiter):
        if math.sqrt(_fdot(r, r)) < atol:
            return x, 0
        z = r if psolve is None else psolve(r)
        rho = _fdot(r, z)
        if it > 0:
            p *= rho / rho_prev
            p += z
        else:
            p = z.copy()
        q = matvec(p)
        alpha = rho / _fdot(p, q)
        x += alpha * p
        r -= alpha * q
        rho_prev = rho
        if callback:
            callback(x)
    return x, maxiter


@pytest.fixture
def exact_cg():
    orig = O.scipy_cg
    O.scipy_cg = scipy_cg_exact
    yield
    O.scipy_cg = orig


def test_sensitivity_fixture_is_consistent():
    """Every recorded envelope is the per-iteration maximum of its variants, and every case the GPU
    tests read is present."""
    s = T.sensitivity()
    for name, c in s.items():
        for key in ("x", "r"):
            env = np.asarray(c["envelope"].get(key, []))
            if env.size:
                vmax = np.max([np.asarray(v[key][:env.size]) for v in c["variants"].values() if key in v], axis=0)
                np.testing.assert_array_equal(env, vmax)
            if "diameter" in c:
                # the spread of the signed distances (the reference at 0 included) covers the envelope
                dia = np.asarray(c["diameter"][key])
                sg = np.array([v[key + "s"][:dia.size] for v in c["variants"].values() if key + "s" in v])
                np.testing.assert_allclose(dia, np.maximum(sg.max(0), 0) - np.minimum(sg.min(0), 0), rtol=1e-15)
    need = ["c2_res_old", "c2_res_new", "head8192", "bratu100_r20_res_old", "bratu100_r20_res_new",
            "short256_r3_res_old", "short256_r7_res_old", "short256_r5_res_new"] + \
        [f"multislab{N}_{v}" for N in (256, 384) for v in ("res_old", "res_new", "jac_old_res_old", "jac_old_res_new")] + \
        ["mispredict1024", "gn256", "gn256_pre", "gn384_pre"]
    assert not [n for n in need if n not in s]


@pytest.mark.parametrize("case", ["short256_r3_res_old"])
def test_sensitivity_envelope_recomputed_live(case):
    """The cheap envelopes recomputed here agree with the committed file (same variants)."""
    live = MS.CASES[case]()
    rec = T.sensitivity()[case]
    env_l, env_r = np.asarray(live["envelope"]["x"]), np.asarray(rec["envelope"]["x"])
    assert env_l.shape == env_r.shape
    big = env_r > 1e-13
    np.testing.assert_allclose(env_l[big], env_r[big], rtol=0.5)


def test_k1_step_is_cancellation_limited():
    """C2's first step: ||x_1|| = |c + d| with c = ||x_0|| ~ 123 and d ~ -123 cancels to 2.2e-4; the
    reference's own value (its fixture) is >= 3e-10 away from the step with exactly rounded sums, and
    the recorded envelope at iteration 1 covers it."""
    prob, y, u0 = O.bratu_workload(1024)
    J = prob.make_jac()(u0)
    c = np.linalg.norm(u0)
    v = u0 / c
    r0 = prob.make_res(y)(v * c)
    Jv = J @ v
    x1_exact = abs(c - math.fsum(Jv * r0) / math.fsum(Jv * Jv))
    ref = json.load(open(os.path.join(GOLDEN, "large_c2.json")))["cases"]["res_old"]["per_iter"]["xnorm"][0]
    spread = abs(ref - x1_exact) / x1_exact
    assert spread >= 3e-10
    assert T.per_iteration("c2_res_old", 1)[0] >= 0.9 * spread


def test_exact_dot_cg_reproduces_reference(golden, exact_cg):
    """With exactly rounded dot products (what the device's compensated sums deliver) the reference's
    CG recurrence gives the reference's iteration counts for every golden Bratu solve -- so the GPU
    tests require cg_iter exactly -- and iterates within 1e-10 (GN N = 100: 2.4e-12)."""
    meta, arr = golden
    prob = O.BratuPdeProblem(101, 5, 10)
    y = prob.pde_operator(prob.u_true)
    rec = []
    with contextlib.redirect_stdout(io.StringIO()):
        O.gauss_newton(prob.make_res(y), arr["bratu100_u0"], prob.make_jac(),
                       callback=lambda x, nfev, cg_iter: rec.append((np.linalg.norm(x), cg_iter)))
    ref = meta["cases"]["bratu100_gn"]["per_iter"]
    assert [c for _, c in rec] == ref["cg_iter"]
    np.testing.assert_allclose([x for x, _ in rec], ref["xnorm"], rtol=T.NORTH_STAR)
    for N in (24, 100):
        p2, y2, u2 = O.bratu_workload(N)
        r0, J0 = p2.make_res(y2)(u2), p2.make_jac()(u2)
        for pre, rtol in ((False, 1e-4), (True, 1e-4), (True, 1e-8)):
            name = f"cgls{N}_pre{int(pre)}" + ("_rtol1e-8" if rtol == 1e-8 else "")
            _, it = O.cg_least_squares(-1 * J0, r0, cg_rtol=rtol, preconditioner=pre)
            assert it == meta["cases"][name]["cg_iter"], name


def test_long_cgls_exact_dot_spread(golden, exact_cg):
    """The 949-iteration Jacobi CGLS at N = 100, rtol 1e-8: the exactly rounded recurrence ends
    >= CGLS_LONG_X (of max |x|) away from the reference's np.dot recurrence."""
    meta, arr = golden
    prob, y, u0 = O.bratu_workload(100)
    x, it = O.cg_least_squares(-1 * prob.make_jac()(u0), prob.make_res(y)(u0), cg_rtol=1e-8, preconditioner=True)
    xr = arr["cgls100_pre1_rtol1e-8__x"]
    assert it == 949
    assert np.abs(x - xr).max() / np.abs(xr).max() >= T.CGLS_LONG_X


def test_rosen2_last_cg_count_is_a_tie(golden, exact_cg):
    """Rosenbrock p = 2 GN from (2, 2): with exactly rounded dots the last outer step's CG takes 4
    iterations where the reference's np.dot takes 3 -- the stopping test on a 2-element residual is a
    rounding tie, so the GPU test allows +-1 on that step only."""
    meta, arr = golden
    res, jac = O.rosenbrock(2)
    rec = []
    with contextlib.redirect_stdout(io.StringIO()):
        O.gauss_newton(res, np.array([2.0, 2.0]), jac, callback=lambda x, nfev, cg_iter: rec.append(cg_iter))
    ref = meta["cases"]["rosen2_2_2_gn"]["per_iter"]["cg_iter"]
    assert rec[:-1] == ref[:-1] and abs(rec[-1] - ref[-1]) == 1


def test_c2_res_old_converged_step_is_a_rounding_tie():
    """The reason C2 res_old's last Armijo count is a family of values (tests/tolerances.py): in the reference's
    own run (the pinned oracle, one BLAS thread) the converged step's threshold 0.5 t ||J d||^2 is a fraction
    of one ulp of the loss, so each trial's test prev - cur >= 0.5 t ||J d||^2 (ref:armijo_goldstein.py:57-62)
    is decided by the rounding of the two sums of squares; its trials sit a few ulps from prev."""
    prob, y, u0 = O.bratu_workload(1024)
    rec = []
    orig = O.armijo_goldstein

    def arm(res, x, res_ev, jac_ev, args, d, max_iter=100, initial_step_length=1.0):
        prev, jdd = np.sum(res_ev ** 2), np.sum((jac_ev @ d) ** 2)
        out = orig(res, x, res_ev, jac_ev, args, d, max_iter, initial_step_length)
        t, losses = 1.0, []
        for _ in range(out[2]):
            losses.append(np.sum(res(x + t * d) ** 2))
            t /= 2
        rec.append((prev, jdd, losses))
        return out

    O.armijo_goldstein = arm
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            O.gauss_newton_krylow(prob.make_res(y), u0, prob.make_jac(), krylow_restart=20, max_iter=100,
                                  version="res_old")
    finally:
        O.armijo_goldstein = orig
    prev, jdd, losses = rec[-1]
    ulp = np.finfo(np.float64).eps * prev
    assert 0.5 * jdd < 0.1 * ulp
    assert all(abs(prev - c) <= T.ARMIJO_TIE_ULPS * ulp for c in losses)
    assert len(losses) == 2                       # the reference's own count for this step (83 - 81)
