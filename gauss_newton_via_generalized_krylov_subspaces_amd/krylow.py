"""Generalized Krylov subspace on the GPU (ref:krylow.py:1-73).

The basis is a device matrix ``V`` of shape (kmax, slab_len): row j is basis
column j as a slab vector (column-major basis, contiguous columns), so one
kernel pass streams k contiguous columns.  Columns are appended in place --
the reference's ``np.hstack`` copy of the whole basis (ref:krylow.py:73, 6 % of
its run time) does not exist here.

Numerics follow the reference step by step: single classical Gram-Schmidt
pass (CGS1, :64), breakdown when every |g_i| <= 1e-8 (:66, np.allclose with
rtol=0), normalisation by the 2-norm (:71).

Deferred Gram-Schmidt (the schedule, not the arithmetic, differs from the
reference).  ``update`` computes g = -J^T r and h = V^T g (:62, :64) and stores
the raw g as column k -- the *pending* column -- with its projection
coefficients; it does not stream V a second time for g -= V h.  The pending
column is settled by the next pass that reads V anyway:
  * the next least-squares pass sees J w = J g - (J V) h through its triangular
    transform (lls.py: ``gram_left``);
  * the next first Armijo trial point materialises w = g - V h in place over
    column k (the arithmetic of the CGS kernel) and returns sum w^2 and max |w|
    with the trial's residual, so the norm (:71) and the breakdown test (:66)
    come back with a host read the trial makes anyway (``resolve``);
  * a restart settles it inside the GEMV of the restart point (``x_settle``: the same
    materialisation kernel with coefficient 0 for the column), the end of the loop
    explicitly (``resolve_explicit``).
Column j of the reference basis is ``sc[j] * V[j]`` (sc = 1 / ||w||: the
division of :71 is folded into the coefficients of every product with V).  The
solver keeps the iterate's coordinates twice: ``c`` in the reference's units (the
convergence test, ref:gauss_newton_krylow.py:96-104) and ``e`` in stored units,
e = c * sc as it was accumulated -- every trial point is V @ (e + t ds) and the
accepted one becomes the new e, so the reference's bit identity "the accepted
trial point V (c + t d) is the next iterate V c"  holds for V @ e.
"""
from __future__ import annotations

import math

import numpy as np


class GeneralizedKrylowSubspaceBreakdown(Exception):
    """ref:krylow.py:8-9"""


class GeneralizedKrylowSubspaceSpansEntireSpace(Exception):
    """ref:krylow.py:12-13"""


BREAKDOWN_MESSAGE = ("Normal residual is allready inside generalized Krylow Subspcae, there for gauss newton "
                     "krylow algorithm has to proceed without enlarging the subspace.")


def is_breakdown(sumsq: float, maxabs: float) -> bool:
    """np.allclose(g, 0, atol=1e-8, rtol=0) of ref:krylow.py:66 (NaN is never close)."""
    return maxabs <= 1e-8 and not math.isnan(sumsq)


FUSE_KMAX_NARROW = 24               # k_gemv_vjpg: a point's basis row in VGPRs
FUSE_KMAX_WIDE = 208                # k_trial_w: tiles of the basis through LDS (N % 128 == 0, no segments)


class DeviceKrylovBasis:
    deferred = True

    def __init__(self, dev, kmax: int):
        self.dev = dev
        self.be = dev.backend
        self.kmax = int(kmax)
        # columns the first-trial kernel with the update products covers (gnk_basis_gemv_vjp_gemv_t*): the
        # narrow register kernel up to 24, the wide LDS kernel beyond when the grid allows it
        wide = dev.slab.N % 128 == 0 and not getattr(dev, "seg_rows", 0)
        self.FUSE_KMAX = FUSE_KMAX_WIDE if wide else FUSE_KMAX_NARROW
        self.V = self.be.zeros(self.kmax, dev.slab.length)
        self.k = 0                       # settled columns
        self.sc = np.ones(self.kmax)     # reference column j = sc[j] * V[j]
        self.pend = None                 # pending column: {"slot", "hh", "it"}
        self.last_norm = None            # ||w|| of the column settled last
        self._c = self.be.zeros(self.kmax + 1)
        self._hh = self.be.zeros(self.kmax)
        self._h = self.be.zeros(self.kmax + 1)
        self._stats = self.be.zeros(2)
        self._stats2 = self.be.zeros(4)                   # x_settle_start: [sum w^2, max |w|, sum x^2, max |x|]
        # [sum r^2, sum w^2, max |w|, h_0 .. h_k] of a first trial: one collective / host read (the
        # speculative next step reads it on the device before the next trial overwrites it, in
        # stream order)
        self.pack = self.be.zeros(3 + self.kmax + 1)
        self._sc_dev = [self.be.zeros(self.kmax) for _ in range(2)]      # k_lls_next inputs, per buffer set
        self._g = dev.vec()              # raw g when V has no free slot (never pending in a Gram)

    @property
    def shape(self):
        """(n, k) like ``basis.shape`` in the reference (n = global unknowns, settled columns)."""
        return (self.dev.slab.n_global, self.k)

    @property
    def pending(self) -> bool:
        return self.pend is not None

    def gram_k(self) -> int:
        """Columns the least-squares pass covers: the settled ones and a pending one."""
        return self.k + (1 if self.pend is not None else 0)

    def gram_left(self):
        """Upper-triangular M with [reference columns | w] = [V_0 .. V_{k-1} | g] M: diag(sc) on the
        settled columns and (-hh, 1) in the pending column; None when M = I."""
        k = self.k
        if self.pend is None:
            return None if np.all(self.sc[:k] == 1.0) else np.diag(self.sc[:k])
        M = np.zeros((k + 1, k + 1))
        M[np.arange(k), np.arange(k)] = self.sc[:k]
        M[:k, k] = -self.pend["hh"]
        M[k, k] = 1.0
        return M

    def _slot(self, j):
        return self.V[j] if j < self.kmax else self._g

    def step_scale(self) -> np.ndarray:
        """Per-column factor from a least-squares step to stored units (ds = step_scale * d): sc on
        the settled columns, 1 on a pending one (its step is already in raw units)."""
        return np.append(self.sc[:self.k], 1.0) if self.pend is not None else self.sc[:self.k].copy()

    def start(self, x, stats=None):
        """ref:krylow.py:30-39.  ``x`` is a slab vector valid on owned +-GHOST rows; returns [||x||].
        ``stats``: x's rank-summed (sum x^2, max |x|), already read (``x_settle_start``)."""
        if stats is None:
            self.be.vec_stats(x, self._stats)
            sumsq, maxabs = self.dev.comm.sum_max(self._stats)
        else:
            sumsq, maxabs = stats
        if maxabs <= 1e-8:                                    # np.allclose(x0, 0) (:31)
            raise ValueError("x0 is not allowed to be 0 in the gauss_newton_krylow algorithm")
        nrm = math.sqrt(sumsq)                                # np.linalg.norm (:36)
        self.be.vec_div(x, nrm, self.V[0], True)              # whole slab incl. ghosts (:37)
        self.k = 1
        self.sc[:] = 1.0
        self.pend = None
        return np.array([nrm])

    def x(self, e: np.ndarray, out):
        """out = V @ e over the whole slab (ref:krylow.py:41-42), e in stored units, len(e) <= k."""
        k = len(e)
        if k > self.k:
            raise RuntimeError("basis.x: coefficient vector longer than the settled basis")
        self.be.upload(self._c, e)
        self.be.gemv(self.V, k, self._c, out)
        return out

    # -- first Armijo trial --------------------------------------------------------------
    def enqueue_trial(self, k, pend, out, coef_dev, hh_dev, pack, r_products=None):
        """First trial point on an explicit basis size (no host state read): k settled columns plus,
        when ``pend``, the pending raw column k, materialised in place with the device coefficients
        hh_dev (pack[1:3] = sum w^2, max |w|); out = V @ coef_dev over k + pend columns.  With
        ``r_products``: also g = -J(out)^T r into slot k + pend and pack[3:] = V^T g (this rank).
        Returns the product slot (or None)."""
        kk = k + (1 if pend else 0)
        if r_products is not None:
            if kk > self.FUSE_KMAX:
                raise RuntimeError("fused first trial: too many basis columns")
            g = self._slot(kk)
            h = pack[3:3 + kk]
            if pend:
                self.be.gemv_vjp_gemv_t_pending(self.V, k, coef_dev, hh_dev, r_products, out, g, h, pack[1:3])
            else:
                self.be.gemv_vjp_gemv_t(self.V, kk, coef_dev, r_products, out, g, h)
            return kk
        if pend:
            self.be.gemv_pending(self.V, k, coef_dev, hh_dev, out, pack[1:3])
        else:
            self.be.gemv(self.V, kk, coef_dev, out)
        return None

    def halo_slot(self, j):
        """Exchange the ghost rows of stored column j (a raw g the next pass reads off-rank)."""
        self.dev.comm.halo(self._slot(j), self.dev.slab.N, self.dev.slab.nrows)

    def sc_device(self, par, k):
        """The folded column scales sc[:k] uploaded into device buffer ``par`` (k_lls_next input)."""
        self.be.upload(self._sc_dev[par], self.sc[:k])
        return self._sc_dev[par]

    def trial_first(self, e_ext, out, r_products=None, coef_dev=None, pack=None, hh_dev=None):
        """``enqueue_trial`` on the host's current basis (settled k, pending column if any; its hh
        uploaded, or ``hh_dev``: the same coefficients already on the device -- an adopted speculative
        solve's), coefficients e_ext (host, stored units) or ``coef_dev``.  Returns (pack, slot)."""
        pack = self.pack if pack is None else pack
        kk = self.gram_k()
        if coef_dev is None:
            if len(e_ext) != kk:
                raise RuntimeError("trial_first: coefficient length != basis columns")
            self.be.upload(self._c, e_ext)
            coef_dev = self._c
        elif coef_dev.numel() < kk:
            raise RuntimeError("trial_first: device coefficients shorter than the basis")
        pend = self.pend is not None
        if pend:
            if self.pend["slot"] != self.k:
                raise RuntimeError("pending column is not stored in V")
            if hh_dev is None or hh_dev.numel() != len(self.pend["hh"]):
                self.be.upload(self._hh, self.pend["hh"])
                hh_dev = self._hh
        slot = self.enqueue_trial(self.k, pend, out, coef_dev, hh_dev, pack, r_products)
        return pack, slot

    def resolve(self, sumsq: float, maxabs: float) -> bool:
        """Settle the pending column from its materialisation stats; True on breakdown (:66) --
        then the column is dropped, else it becomes column k with sc = 1 / ||w|| (:71)."""
        self.pend = None
        if is_breakdown(sumsq, maxabs):
            self.last_norm = None
            return True
        nrm = math.sqrt(sumsq)
        self.last_norm = nrm
        self.sc[self.k] = 1.0 / nrm
        self.k += 1
        return False

    def resolve_explicit(self) -> bool:
        """Settle a pending column without a trial (restart / end of the loop): w = g - V hh in place on
        owned rows, then ``resolve``.  (Ghost rows are not refreshed: the caller discards the column.)"""
        g = self._slot(self.pend["slot"])
        self.be.upload(self._hh, self.pend["hh"])
        self.be.cgs_update(self.V, self.k, self._hh, g, self._stats)
        sumsq, maxabs = self.dev.comm.sum_max(self._stats)
        return self.resolve(sumsq, maxabs)

    def x_settle(self, e: np.ndarray, out) -> bool:
        """Restart point out = V @ e (e over the k settled columns, the reference's V @ c) with the
        pending column settled in the same pass: k_gemv_p materialises w = g - V hh and returns
        sum w^2, max |w| for its breakdown test (ref:krylow.py:66) -- the column itself enters out with
        coefficient 0, as the reference's appended coordinate.  Replaces cgs_update + gemv (one read
        of V instead of two).  Returns True on breakdown (then the column is dropped)."""
        k = self.k
        if self.pend is None or self.pend["slot"] != k:
            raise RuntimeError("x_settle: no pending column in slot k")
        if len(e) != k:
            raise RuntimeError("x_settle: coefficient vector must cover the settled columns")
        self.be.upload(self._c, np.append(e, 0.0))
        self.be.upload(self._hh, self.pend["hh"])
        self.be.gemv_pending(self.V, k, self._c, self._hh, out, self._stats)
        sumsq, maxabs = self.dev.comm.sum_max(self._stats)
        return self.resolve(sumsq, maxabs)

    def x_settle_start(self, e: np.ndarray, out):
        """``x_settle`` with the stats ``start`` needs of its result read back in the same host read: the
        restart point out = V @ e does not depend on the pending column's breakdown decision (the column
        enters with coefficient 0), so its sum x^2 / max |x| (the kernel ``start`` would launch next) are
        enqueued behind the settling GEMV and both [sum, max] pairs come back in one collective.  The same
        kernels and the same rank combine as x_settle then start: bit for bit.  Returns (breakdown,
        (sum x^2, max |x|)) -- pass the latter to ``start``."""
        k = self.k
        if self.pend is None or self.pend["slot"] != k:
            raise RuntimeError("x_settle_start: no pending column in slot k")
        if len(e) != k:
            raise RuntimeError("x_settle_start: coefficient vector must cover the settled columns")
        self.be.upload(self._c, np.append(e, 0.0))
        self.be.upload(self._hh, self.pend["hh"])
        self.be.gemv_pending(self.V, k, self._c, self._hh, out, self._stats2[0:2])
        self.be.vec_stats(out, self._stats2[2:4])
        (sw, mw), xs = self.dev.comm.sum_max_pairs(self._stats2, 2)
        return self.resolve(sw, mw), xs

    # -- basis update ------------------------------------------------------------------------
    def update(self, u_jac, r, it=None, products=None, prod_slot=None, halo=True):
        """ref:krylow.py:55-73 with jac_ev = J(u_jac), res_ev = r (slab vectors), deferred: the new
        column becomes pending (see the module docstring).  ``products``: the rank-summed raw
        h = V^T g already computed at u_jac with residual r, g in slot ``prod_slot``; ``halo``:
        False when g's ghost rows were already exchanged (a speculative next step did it)."""
        k = self.k
        if self.pend is not None:
            raise RuntimeError("basis update with a pending column")
        if k == self.dev.slab.n_global:                       # :59-60
            raise GeneralizedKrylowSubspaceSpansEntireSpace
        if k >= self.kmax:
            raise RuntimeError("Krylov basis storage exhausted")
        g = self._slot(k)
        if products is not None:
            if prod_slot != k:
                raise RuntimeError("update products were computed for another basis size")
            h_raw = np.asarray(products[:k], dtype=np.float64)
        else:
            self.be.vjp_gemv_t(u_jac, r, self.V, k, g, self._h)       # g = -J^T r ; h = V^T g (:62, :64)
            h_raw = self.dev.comm.sum(self._h[:k])                   # rank-ordered sum of the partials
            halo = True
        # g's ghost rows: the next pass applies the stencil to it and materialises w on the whole slab
        if halo:
            self.dev.comm.halo(g, self.dev.slab.N, self.dev.slab.nrows)
        h = self.sc[:k] * h_raw                                      # reference h = V^T g
        self.pend = {"slot": k, "hh": self.sc[:k] * h, "it": it}
