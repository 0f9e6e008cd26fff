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
