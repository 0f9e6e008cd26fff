"""Projected least-squares solve of the GNK step (ref:gauss_newton_krylow.py:16-36, 89).

The reference factors A = -J @ V (n x k) with LAPACK Householder QR and solves
R d = Q^T r.  The build never materialises J @ V: the fp64-MFMA Gram kernel
(gnk_gram) streams V once per pass, applies the Bratu stencil on the fly, applies
an upper-triangular preconditioner P^-1 on MFMA (W <- W P^-1) and returns the Gram
matrix of [J V P^-1 | r].  Cholesky QR on a well-conditioned Y = J V P^-1 gives
R = R_Y P and Q^T r = R_Y^-T (Y^T r) to O(u) orthogonality.

Preconditioner P (one pass per iteration in the common case):
  * CholQR2 (two passes: P = I, then P = R1) when there is no usable previous
    factor and no column scale (after a breakdown-free restart the solver passes
    s = ||J v_0|| and the first solve is a single pass with P = [s]);
  * otherwise P = blockdiag(R_prev, s): the previous iteration's R of J_prev V
    (the basis only gained one column and J changed only in its diagonal
    LAMBDA exp(u)) and s = ||J v_new|| for the appended column, so Y is close to
    orthonormal and ONE pass suffices.
The pass is accepted when cond(R_Y) <= COND_ACCEPT (then the O(cond^2 u)
CholQR error is below 1e-13 relative); otherwise another pass runs with the
current R -- classical CholQR2 -- and, if a Gram is not numerically SPD, the
factorisation is shifted (shifted CholeskyQR3, Fukaya et al. 2020).
Across ranks each Gram is an all-gather of (k+1)^2 doubles summed in rank order
(the "one-reduce" of TSQR, once per pass).

jdd = ||J V d||^2 of the Armijo rule (ref:armijo_goldstein.py:50) is ||R d||^2:
the reference's extra GEMV over J V is not needed.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

EPS = np.finfo(np.float64).eps
COND_ACCEPT = 30.0
MAX_PASSES = 4


def _chol_upper(G):
    R = scipy.linalg.cholesky(G, lower=False, check_finite=False)
    if not np.all(np.isfinite(R)):
        raise np.linalg.LinAlgError("non-finite Cholesky factor")
    return R


def _cond_upper(R):
    d = np.abs(np.diagonal(R))
    if d.min() == 0.0:
        return np.inf
    return float(np.linalg.cond(R))


class CholQR2Solver:
    def __init__(self, dev, kmax: int, gram=None, n_global=None):
        """``gram(u, V, k, rinv, r, G)`` fills G with the Gram of [J(u) V RinvAug | r] (default:
        the Bratu stencil kernel); ``n_global`` = parameter count (for the sCholQR3 shift)."""
        self.dev = dev
        self.be = dev.backend
        self._gram_fn = gram if gram is not None else self.be.gram
        self.n_global = n_global if n_global is not None else dev.slab.n_global
        kp = self.be.gram_dim(kmax, True)
        self._G = self.be.zeros(kp * kp)
        self._rinv = self.be.zeros(kp * kp)
        self.passes = 0
        self.solves = 0
        self.fallbacks = 0
        self.history = []           # per solve: (k, passes, cond(R_Y) of each pass) -- diagnostics
        self.R_prev = None          # R of the last solve (k_prev x k_prev); None after a restart
        self.R_last = None          # R of the last solve (diagnostics)
        self.s_new = None           # ||J v_new|| of the column appended since then

    # -- basis events (the solver tells us how V changed since the last solve) -------
    def on_append(self, s_new):
        """s_new = ||J v_new||, a float or a callable returning it (read lazily at the next solve)."""
        self.s_new = s_new

    def on_restart(self, s0=None):
        """The basis restarted with one column v_0; s0 = ||J v_0|| (None: unknown -> CholQR2)."""
        self.R_prev = None if s0 is None else np.zeros((0, 0))
        self.s_new = s0

    def _gram(self, u, basis, k, P, r):
        be = self.be
        kp = be.gram_dim(k, r is not None)
        rinv_dev = None
        if P is not None:
            aug = np.zeros((kp, kp))
            aug[:k, :k] = scipy.linalg.solve_triangular(P, np.eye(k), lower=False)
            if r is not None:
                aug[k, k] = 1.0
            rinv_dev = self._rinv[:kp * kp]
            be.upload(rinv_dev, aug.reshape(-1))
        G = self._G[:kp * kp]
        self._gram_fn(u, basis.V, k, rinv_dev, r, G)
        self.passes += 1
        return self.dev.comm.sum(G).reshape(kp, kp)

    def _initial_preconditioner(self, k):
        R = self.R_prev
        if R is None:
            return None
        if callable(self.s_new):
            self.s_new = float(self.s_new())
        kp = R.shape[0]
        if kp == k:
            return R                                   # basis unchanged (breakdown / spans space)
        if kp == k - 1 and self.s_new is not None and self.s_new > 0.0:
            P = np.zeros((k, k))
            P[:kp, :kp] = R
            P[kp, kp] = self.s_new
            return P
        return None

    def solve(self, u, basis, r):
        """Returns (d, jdd, R) for min ||-J(u) V d - r||."""
        k = basis.k
        self.solves += 1
        p0 = self.passes
        conds = []
        P = self._initial_preconditioner(k)
        if P is None:
            # classical CholQR2: first pass unpreconditioned (P = I, no r column)
            G1 = self._gram(u, basis, k, None, None)[:k, :k]
            try:
                P = _chol_upper(G1)
            except (np.linalg.LinAlgError, ValueError):
                n = self.n_global
                shift = 11.0 * (n * k + k * (k + 1)) * EPS * np.trace(G1)
                P = _chol_upper(G1 + shift * np.eye(k))
        for it in range(MAX_PASSES):
            Gp = self._gram(u, basis, k, P, r)
            try:
                Ry = _chol_upper(Gp[:k, :k])
            except (np.linalg.LinAlgError, ValueError):
                n = self.n_global
                shift = 11.0 * (n * k + k * (k + 1)) * EPS * np.trace(Gp[:k, :k])
                P = _chol_upper(Gp[:k, :k] + shift * np.eye(k)) @ P
                self.fallbacks += 1
                continue
            conds.append(_cond_upper(Ry))
            if conds[-1] <= COND_ACCEPT or it == MAX_PASSES - 1:
                z = scipy.linalg.solve_triangular(Ry, Gp[:k, k], trans="T", lower=False)
                R = Ry @ P
                break
            P = Ry @ P                                   # one more pass with the improved factor
            self.fallbacks += 1
        for r_kk in np.diagonal(R):                                  # ref:gauss_newton_krylow.py:32-34
            if np.isclose(r_kk, 0, atol=1e-8):
                print("A is rank deficient")
        d = -scipy.linalg.solve_triangular(R, z, lower=False)
        jdd = float(np.sum((R @ d) ** 2))
        self.history.append((k, self.passes - p0, conds))
        self.R_prev = self.R_last = R
        self.s_new = None
        return d, jdd, R
