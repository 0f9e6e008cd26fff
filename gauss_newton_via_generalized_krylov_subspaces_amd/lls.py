"""Projected least-squares solve of the GNK step (ref:gauss_newton_krylow.py:16-36, 89).

The reference factors A = -J @ V (n x k) with LAPACK Householder QR and solves
R d = Q^T r.  The build never materialises J @ V: the fp64-MFMA Gram kernel
(gnk_gram) streams V once per pass, applies the Bratu stencil on the fly and
returns W^T W.  CholeskyQR2 on those Gram matrices gives the same R (up to row
signs) and Q^T r to O(u) orthogonality for cond(J V) up to ~1e7:

  pass 1:  G1 = (J V)^T (J V)                      -> R1 = chol(G1)
  pass 2:  G2 = [J V R1^-1 | r]^T [J V R1^-1 | r]   -> R2 = chol(G2[:k,:k]),
           z = R2^-T G2[:k, k] = Q^T r,  R = R2 R1,  d = -R^-1 z.

If pass 1 is not numerically SPD the first factorisation is shifted
(shifted CholeskyQR3, Fukaya et al. 2020) and one more pass is made.
Across ranks each Gram is an all-gather of (k+1)^2 doubles summed in rank order
(the "one-reduce" of TSQR, once per pass).

jdd = ||J V d||^2 of the Armijo rule (ref:armijo_goldstein.py:50) is ||R d||^2:
the reference's extra GEMV over J V is not needed.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg

EPS = np.finfo(np.float64).eps


def _chol_upper(G):
    return scipy.linalg.cholesky(G, lower=False, check_finite=False)


class CholQR2Solver:
    def __init__(self, dev, kmax: int):
        self.dev = dev
        self.be = dev.backend
        kp = self.be.gram_dim(kmax, True)
        self._G = self.be.zeros(kp * kp)
        self._rinv = self.be.zeros(kp * kp)
        self.passes = 0

    def _gram(self, u, basis, k, rinv_host, r):
        be = self.be
        kp = be.gram_dim(k, r is not None)
        rinv_dev = None
        if rinv_host is not None:
            aug = np.zeros((kp, kp))
            aug[:k, :k] = rinv_host
            if r is not None:
                aug[k, k] = 1.0
            rinv_dev = self._rinv[:kp * kp]
            rinv_dev.copy_(be.to_device(aug.reshape(-1)))
        G = self._G[:kp * kp]
        be.gram(u, basis.V, k, rinv_dev, r, G)
        self.passes += 1
        return self.dev.comm.sum(G).reshape(kp, kp)

    def solve(self, u, basis, r):
        """Returns (d, jdd, R) for min ||-J(u) V d - r||."""
        k = basis.k
        G1 = self._gram(u, basis, k, None, None)[:k, :k]
        shifted = False
        try:
            R = _chol_upper(G1)
            if not np.all(np.isfinite(R)):
                raise np.linalg.LinAlgError
        except (np.linalg.LinAlgError, ValueError):
            n = self.dev.slab.n_global
            s = 11.0 * (n * k + k * (k + 1)) * EPS * np.trace(G1)
            R = _chol_upper(G1 + s * np.eye(k))
            shifted = True
        npass = 3 if shifted else 2
        for p in range(1, npass):
            last = p == npass - 1
            Rinv = scipy.linalg.solve_triangular(R, np.eye(k), lower=False)
            Gp = self._gram(u, basis, k, Rinv, r if last else None)
            Rp = _chol_upper(Gp[:k, :k])
            if last:
                z = scipy.linalg.solve_triangular(Rp, Gp[:k, k], trans="T", lower=False)
            R = Rp @ R
        for r_kk in np.diagonal(R):                                  # ref:gauss_newton_krylow.py:32-34
            if np.isclose(r_kk, 0, atol=1e-8):
                print("A is rank deficient")
        d = -scipy.linalg.solve_triangular(R, z, lower=False)
        jdd = float(np.sum((R @ d) ** 2))
        return d, jdd, R
