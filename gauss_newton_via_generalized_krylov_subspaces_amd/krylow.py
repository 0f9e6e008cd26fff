"""Generalized Krylov subspace on the GPU (ref:krylow.py:1-73).

The basis is a device matrix ``V`` of shape (kmax, slab_len): row j is basis
column j as a slab vector (column-major basis, contiguous columns), so one
kernel pass streams k contiguous columns.  Columns are appended in place --
the reference's ``np.hstack`` copy of the whole basis (ref:krylow.py:73, 6 % of
its run time) does not exist here.

Numerics follow the reference step by step: single classical Gram-Schmidt
pass (CGS1, :64), breakdown when every |g_i| <= 1e-8 (:66, np.allclose with
rtol=0), normalisation by division (:71).
"""
from __future__ import annotations

import math

import numpy as np


class GeneralizedKrylowSubspaceBreakdown(Exception):
    """ref:krylow.py:8-9"""


class GeneralizedKrylowSubspaceSpansEntireSpace(Exception):
    """ref:krylow.py:12-13"""


class DeviceKrylovBasis:
    def __init__(self, dev, kmax: int):
        self.dev = dev
        self.be = dev.backend
        self.kmax = int(kmax)
        self.V = self.be.zeros(self.kmax, dev.slab.length)
        self.k = 0
        self._c = self.be.zeros(self.kmax)
        self._h = self.be.zeros(self.kmax)
        self._stats = self.be.zeros(2)
        self._pack = self.be.zeros(3)          # [residual partial, sum g^2, max |g|] of a speculative step
        self._g = dev.vec()              # new column before normalisation (stencil source)
        self._jn2 = self.be.zeros(1)

    @property
    def shape(self):
        """(n, k) like ``basis.shape`` in the reference (n = global unknowns)."""
        return (self.dev.slab.n_global, self.k)

    def start(self, x, u_jac=None):
        """ref:krylow.py:30-39.  ``x`` is a slab vector valid on owned +-GHOST rows.

        Returns the coordinates [||x||]; with ``u_jac`` also ||J(u_jac) v_0|| (the first
        least-squares preconditioner), from the same pass that normalises x."""
        self.be.vec_stats(x, self._stats)
        sumsq, maxabs = self.dev.comm.sum_max(self._stats)
        if maxabs <= 1e-8:                                    # np.allclose(x0, 0) (:31)
            raise ValueError("x0 is not allowed to be 0 in the gauss_newton_krylow algorithm")
        nrm = math.sqrt(sumsq)                                # np.linalg.norm (:36)
        self.k = 1
        if u_jac is None:
            self.be.vec_div(x, nrm, self.V[0], True)          # whole slab incl. ghosts (:37)
            return np.array([nrm])
        self.be.normalize_jnorm(u_jac, x, nrm, self.V[0], self._jn2)
        return np.array([nrm]), math.sqrt(float(self.dev.comm.sum(self._jn2)[0])) / nrm

    def x(self, c: np.ndarray, out):
        """out = V @ c over the whole slab (ref:krylow.py:41-42)."""
        k = len(c)
        self.be.upload(self._c, c)
        self.be.gemv(self.V, k, self._c, out)
        return out

    FUSE_KMAX = 24

    def x_with_update_products(self, c: np.ndarray, r, out):
        """out = V @ c, and -- from the same read of V -- the products of a basis update at
        u = out with residual r: g = -J(out)^T r, h = V^T g (this rank's rows).  ``update(...,
        products_ready=True)`` then continues from them.  Used for the first Armijo trial of
        version "res_old" (the update after acceptance is exactly this product)."""
        k = len(c)
        self.be.upload(self._c, c)
        self.be.gemv_vjp_gemv_t(self.V, k, self._c, r, out, self._g, self._h)
        return out

    def cgs_speculative(self):
        """Right after ``x_with_update_products``: enqueue the CGS step g -= V h (+ its stats into
        pack[1:3]) before the Armijo test has read the trial's residual, so that one host read serves
        both (pack[0] is the caller's residual slot).  ``update(..., stats=...)`` continues from it;
        a rejected trial recomputes g."""
        k = self.k
        if self.dev.comm.world > 1:
            self._h[:k].copy_(self.dev.comm.sum_device(self._h[:k]))
        self.be.cgs_update(self.V, k, self._h, self._g, self._pack[1:3])
        return self._pack

    def update(self, u_jac, r, u_next=None, products_ready=False, stats=None):
        """ref:krylow.py:55-73 with jac_ev = J(u_jac), res_ev = r (slab vectors).

        Returns ||J(u_next) v_new|| (u_next defaults to u_jac), computed in the same
        pass that normalises the new column (the next least-squares preconditioner).
        ``products_ready``: g and h were produced by ``x_with_update_products`` at u_jac;
        ``stats`` = (sum g^2, max |g|) when ``cgs_speculative`` has also done the CGS step."""
        k = self.k
        if k == self.dev.slab.n_global:                       # :59-60
            raise GeneralizedKrylowSubspaceSpansEntireSpace
        if k >= self.kmax:
            raise RuntimeError("Krylov basis storage exhausted")
        g = self._g
        if stats is not None and products_ready:
            sumsq, maxabs = stats
        else:
            if not products_ready:
                self.be.vjp_gemv_t(u_jac, r, self.V, k, g, self._h)   # g = -J^T r ; h = V^T g (:62, :64)
            if self.dev.comm.world > 1:                           # rank-ordered sum of the partials
                self._h[:k].copy_(self.dev.comm.sum_device(self._h[:k]))
            self.be.cgs_update(self.V, k, self._h, g, self._stats)   # g -= V h (:64)
            sumsq, maxabs = self.dev.comm.sum_max(self._stats)
        if maxabs <= 1e-8 and not math.isnan(sumsq):          # :66
            raise GeneralizedKrylowSubspaceBreakdown(
                "Normal residual is allready inside generalized Krylow Subspcae, there for gauss newton "
                "krylow algorithm has to proceed without enlarging the subspace.")
        nrm = math.sqrt(sumsq)                                # :71
        self.dev.comm.halo(g, self.dev.slab.N, self.dev.slab.nrows)
        # V[k] = g / nrm on the whole slab (ghost rows divide the neighbours' g, so they
        # equal the neighbours' V[k] rows bit for bit) + sum (J g)^2 on owned rows
        self.be.normalize_jnorm(u_jac if u_next is None else u_next, g, nrm, self.V[k], self._jn2)
        self.k = k + 1
        jn2, comm = self._jn2, self.dev.comm
        # ||J v_new|| is needed only by the next least-squares solve: read it then (after the Gram
        # pass's own sync) instead of stalling the queue here
        return lambda: math.sqrt(float(comm.sum(jn2)[0])) / nrm
