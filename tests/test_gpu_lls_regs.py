"""The device least-squares solve in its two forms -- one entry per thread on 32 x 32 threads (k_lls_2d, the
default) and one wave with a column per lane (k_lls, GNK_TUNE_LLS 1): the same preconditioned-CholeskyQR step (ref:gauss_newton_krylow.py:16-36
restated in lls.py) with the same IEEE operations in the same order, so every output -- status, jdd, the
rescale s, d, R, Ry, R^-1 and the first trial's coefficients -- must agree bit for bit, and for a Gram that is not
numerically SPD the same values with NaN in the same places."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(rng, k, cond, spd=True):
    n = 4 * (k + 1) + 8
    A = rng.standard_normal((n, k + 1)) * np.logspace(0, np.log10(cond), k + 1)
    G = A.T @ A
    if not spd:
        G[k // 2, k // 2] = -abs(G[k // 2, k // 2])
    P = np.triu(rng.standard_normal((k, k)))
    P[np.diag_indices(k)] = np.abs(P[np.diag_indices(k)]) + 1.0
    return G, P, rng.standard_normal(k), rng.standard_normal(k)


def _solve(be, G, kp, k, P, rescale, sdd, e, lls_mode):
    be.set_tuning("lls", lls_mode)
    L = 32
    Gd = torch.zeros(kp * kp, dtype=torch.float64, device=be.device)
    Gd.view(kp, kp)[:k + 1, :k + 1] = torch.from_numpy(G)
    out = torch.full((3 + L + 3 * L * L,), 7.0, dtype=torch.float64, device=be.device)
    et = torch.full((L,), 7.0, dtype=torch.float64, device=be.device)
    be.lls_solve(Gd, kp, k, be.to_device(P.reshape(-1)), rescale, be.to_device(sdd), be.to_device(e), out, et)
    torch.cuda.synchronize()
    be.set_tuning("lls", 0)
    return out.cpu().numpy(), et.cpu().numpy()


@pytest.mark.parametrize("k", [1, 2, 3, 7, 8, 9, 12, 16, 17, 20, 24, 28, 32])
def test_register_solve_bit_identical(k):
    from gauss_newton_via_generalized_krylov_subspaces_amd._native import HipBackend
    be = HipBackend(torch.device("cuda", 0))
    rng = np.random.default_rng(100 + k)
    kp = be.gram_dim(k, True)
    for cond, spd, rescale in ((1e2, True, 1), (1e5, True, 0), (1e3, False, 1), (10.0, True, 1)):
        G, P, sdd, e = _case(rng, k, cond, spd)
        o1, t1 = _solve(be, G, kp, k, P, rescale, sdd, e, 1)
        for mode in (0,):
            o0, t0 = _solve(be, G, kp, k, P, rescale, sdd, e, mode)
            if spd:
                assert o0[0] == 0.0
                assert np.array_equal(o0.view(np.int64), o1.view(np.int64)), (mode, k, cond, rescale)
                assert np.array_equal(t0.view(np.int64), t1.view(np.int64)), (mode, k, cond, rescale)
            else:
                # not SPD: status 1 in all (the host then finishes the solve); the NaNs the factorisation
                # spreads sit in the same places, their sign / payload bits may differ (operand order of
                # NaN propagation), every other value is the same double
                assert o0[0] == o1[0] == 1.0
                assert np.array_equal(o0, o1, equal_nan=True) and np.array_equal(t0, t1, equal_nan=True)
