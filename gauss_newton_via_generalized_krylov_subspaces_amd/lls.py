"""Projected least-squares solve of the GNK step (ref:gauss_newton_krylow.py:16-36, 89).

The reference factors A = -J @ V (n x k) with LAPACK Householder QR and solves
R d = Q^T r.  The build never materialises J @ V: the fp64-MFMA Gram kernel
(gnk_gram) streams the stored basis once per pass, applies the Bratu stencil on
the fly, applies an upper-triangular transform T on MFMA and returns the Gram
matrix of [J V_stored T | r].  Cholesky QR on a well-conditioned Y gives R and
Q^T r = R_Y^-T (Y^T r) to O(u) orthogonality.

T = M P^-1:
  * M (``basis.gram_left()``) maps the stored columns to the reference basis --
    the folded column norms diag(sc) and, for a pending column of the deferred
    Gram-Schmidt (krylow.py), its projection: J w = J g - (J V) hh;
  * P is the preconditioner.  One pass per iteration in the common case:
    P = blockdiag(R_prev, 1) -- the previous iteration's R of J_prev V (the basis
    only gained one column and J changed only in its diagonal LAMBDA exp(u)) --
    and the new column's scale is taken from the same pass: its Gram row/column
    are divided by sqrt(G_kk) (= ||J v_new||), i.e. P = blockdiag(R_prev, ||J v_new||),
    so Y is close to orthonormal.  Without a usable previous factor: CholQR2
    (a plain first pass, P = R_1).
The pass is accepted when cond(R_Y) <= COND_ACCEPT (then the O(cond^2 u) CholQR
error is below 1e-13 relative); otherwise another pass runs with the current R --
classical CholQR2 -- and, if a Gram is not numerically SPD, the factorisation is
shifted (shifted CholeskyQR3, Fukaya et al. 2020).  Across ranks each Gram is an
all-gather of (k+1)^2 doubles summed in rank order (the "one-reduce" of TSQR).

With a pending column the solution is in that column's raw units until the
first trial has measured ||w||: ``resolve_pending(nrm)`` rescales R's last column
and d's last entry to the reference's unit column and only then prints the
rank-deficiency messages; ``discard_pending()`` drops the solve on a breakdown.

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
    sv = np.linalg.svd(R, compute_uv=False)              # 2-norm condition number (np.linalg.cond)
    return float(sv[0] / sv[-1])


def rank_messages(R):
    """ref:gauss_newton_krylow.py:32-34: one message per diagonal entry with np.isclose(r_kk, 0),
    i.e. |r_kk| <= 1e-8 (+ 1e-5 * 0), in diagonal order."""
    for _ in range(int(np.count_nonzero(np.abs(np.diagonal(R)) <= 1e-8))):
        print("A is rank deficient")


class DeviceSolve:
    """A least-squares solve enqueued on the device (``CholQR2Solver.launch``): its first pass and
    the k_lls solve are in the stream; ``out`` / ``e_try`` are device buffers (read with the first
    Armijo trial's scalars, so the Gram -> trial sequence has no host round trip)."""

    device = True

    def __init__(self, k, kp, M, M_cont, P, rescale, pending, G, out, e_try, hh_dev=None, sc_dev=None):
        self.k, self.kp, self.M, self.M_cont, self.P, self.rescale = k, kp, M, M_cont, P, rescale
        self.pending, self.G, self.out, self.e_try = pending, G, out, e_try
        # speculative solves (launch_next): the pending column's projection coefficients hh' and the
        # column scales sc'[:k-1] that k_lls_next formed on the device -- the values the host computes
        # for the same step once it has read the previous one (same IEEE operations on the same
        # inputs), so the step that adopts this solve uses them instead of uploading its own
        self.hh_dev, self.sc_dev = hh_dev, sc_dev


class _LSBuffers:
    """Device inputs / outputs of one device solve; two sets, so that a speculatively enqueued next
    step never overwrites what the host has not read yet."""

    def __init__(self, be, L, kp, pack_room=0):
        self.T = be.zeros(kp * kp)            # augmented transform of the first pass
        self.G = be.zeros(kp * kp)            # its Gram
        self.P = be.zeros(L * L)
        self.sdd = be.zeros(L)
        self.e = be.zeros(L)
        # [the first trial's scalar pack | the solve's output] in one buffer: the step's host read (the
        # pack with the solve) is then one device-to-host copy on one rank
        self.comb = be.zeros(pack_room + 3 + L + 3 * L * L)
        self.pack = self.comb[:pack_room]
        self.out = self.comb[pack_room:]
        self.etry = be.zeros(L)
        self.hh = be.zeros(L)                 # next step's projection coefficients (k_lls_next)
        self.sc = be.zeros(L)


class HostSolve:
    device = False

    def __init__(self, d, jdd):
        self.d, self.jdd = d, jdd


class CholQR2Solver:
    def __init__(self, dev, kmax: int, gram=None, n_global=None, device_solve=True):
        """``gram(u, V, k, rinv, r, G)`` fills G with the Gram of [J(u) V RinvAug | r] (default:
        the Bratu stencil kernel); ``n_global`` = parameter count (for the sCholQR3 shift);
        ``device_solve``: allow ``launch`` to solve on the device (k_lls)."""
        self.dev = dev
        self.be = dev.backend
        self._gram_fn = gram if gram is not None else self.be.gram
        self.n_global = n_global if n_global is not None else dev.slab.n_global
        kp = self.be.gram_dim(kmax, True)
        self._G = self.be.zeros(kp * kp)
        self._rinv = self.be.zeros(kp * kp)
        self.quiet = False          # True: no rank-deficiency messages (GN's lstsq branch prints none)
        self.min_norm_if_singular = False   # True: a singular Gram -> minimum-norm solution (lstsq branch)
        self.passes = 0
        self.solves = 0
        self.fallbacks = 0
        self.device_solves = 0
        self.history = []           # per solve: (k, passes, cond(R_Y) of each pass) -- diagnostics
        self.R_prev = None          # R of the last solve (k_prev x k_prev); None: no usable factor
        self.R_last = None          # R of the last solve (diagnostics)
        self._tentative = None      # (R, d, singular) of a solve over a pending column
        # device solve (k_lls): k <= lsk
        self.lsk = (min(int(self.be.lls_max_k()), int(kmax))
                    if device_solve and hasattr(self.be, "lls_solve") else 0)
        self.pack_room = 4 + int(kmax)          # the basis's first-trial pack (krylow.DeviceKrylovBasis.pack)
        self.bufs = [_LSBuffers(self.be, self.lsk, kp, self.pack_room) for _ in range(2)] if self.lsk else []

    # -- basis events (the solver tells us how V changed since the last solve) -------
    def on_append(self, s_new=None):
        """A column was appended (its scale is measured by the next pass itself)."""

    def on_restart(self, s0=None):
        """The basis restarted with one column v_0: P = [1], scale from the pass."""
        self.R_prev = np.zeros((0, 0))

    def _augment(self, k, T, with_r):
        kp = self.be.gram_dim(k, with_r)
        aug = np.zeros((kp, kp))
        aug[:k, :k] = T
        if with_r:
            aug[k, k] = 1.0
        return aug

    def _gram_device(self, u, basis, k, T, r, T_dev=None, G_dev=None):
        """Enqueue one pass; returns the rank-summed Gram as a device tensor (no host read).
        ``T_dev``: the augmented transform already on the device; ``G_dev``: output buffer."""
        kp = self.be.gram_dim(k, r is not None)
        rinv_dev = T_dev[:kp * kp] if T_dev is not None else None
        if T is not None and T_dev is None:
            rinv_dev = self._rinv[:kp * kp]
            self.be.upload(rinv_dev, self._augment(k, T, r is not None).reshape(-1))
        G = (G_dev if G_dev is not None else self._G)[:kp * kp]
        self._gram_fn(u, basis.V, k, rinv_dev, r, G)
        self.passes += 1
        return self.dev.comm.sum_device(G)

    def _gram(self, u, basis, k, T, r):
        kp = self.be.gram_dim(k, r is not None)
        G = self._gram_device(u, basis, k, T, r)
        return G.to("cpu").numpy().reshape(kp, kp).copy()

    def _initial_preconditioner(self, k):
        """(P, rescale_last): P = R_prev (basis unchanged) or blockdiag(R_prev, 1) (one new column,
        scaled by the pass); (None, False) -> CholQR2."""
        R = self.R_prev
        if R is None:
            return None, False
        kp = R.shape[0]
        if kp == k:
            return R, False                            # basis unchanged (breakdown / spans space)
        if kp == k - 1:
            P = np.zeros((k, k))
            P[:kp, :kp] = R
            P[kp, kp] = 1.0
            return P, True
        return None, False

    @staticmethod
    def _transform(M, P):
        Pinv = scipy.linalg.solve_triangular(P, np.eye(P.shape[0]), lower=False)
        return Pinv if M is None else M @ Pinv

    # -- device solve ------------------------------------------------------------------------
    def launch(self, u, basis, r, e_ext, sdd, par=0):
        """Start the solve of min ||-J(u) V d - r||.  When the device can take it (a usable
        preconditioner and k <= lsk): enqueue the first pass and k_lls, which also forms the first
        trial's coefficients e_try = e_ext + sdd * d on the device -> DeviceSolve.  Otherwise solve
        on the host -> HostSolve (d, jdd; tentative when a column is pending)."""
        k = basis.gram_k() if hasattr(basis, "gram_k") else basis.k
        P, rescale = self._initial_preconditioner(k)
        if P is None or k > self.lsk:
            d, jdd, _ = self.solve(u, basis, r)
            return HostSolve(d, jdd)
        M = basis.gram_left() if hasattr(basis, "gram_left") else None
        pending = getattr(basis, "pending", False)
        if pending:
            # after the first trial settles the column, its stored vector is w in the units this solve
            # uses: further passes (continue_host) map it with 1, not sc
            M_cont = np.diag(np.append(basis.sc[:k - 1], 1.0))
        else:
            M_cont = M
        self.solves += 1
        self.device_solves += 1
        P = P.copy()
        B = self.bufs[par]
        G = self._gram_device(u, basis, k, self._transform(M, P), r, G_dev=B.G)
        be = self.be
        be.upload(B.P, P.reshape(-1))
        be.upload(B.sdd, np.asarray(sdd, dtype=np.float64))
        be.upload(B.e, np.asarray(e_ext, dtype=np.float64))
        kp = be.gram_dim(k, True)
        be.lls_solve(G, kp, k, B.P, rescale, B.sdd, B.e, B.out, B.etry)
        return DeviceSolve(k, kp, M, M_cont, P, rescale, pending, G, B.out[:3 + k + 3 * k * k], B.etry[:k])

    def launch_next(self, u, basis, r, ls: "DeviceSolve", pack_sum, sc_dev, par):
        """Speculative device solve of the NEXT step, enqueued before the host has read this one:
        assumes this step (``ls``, pending column or not) accepts its first trial and the basis update
        appends a pending column with the products in ``pack_sum`` (k_lls_next builds T, P, sdd, e and
        hh on the device).  The host fields of the returned DeviceSolve (M, M_cont, P) are filled by
        ``adopt`` once the host state has caught up."""
        k = ls.k + 1
        B = self.bufs[par]
        kp = self.be.gram_dim(k, True)
        self.be.lls_next(ls.k, ls.pending, ls.out, ls.e_try, pack_sum, sc_dev, kp, B.T, B.P, B.sdd, B.e, B.hh, B.sc)
        G = self._gram_device(u, basis, k, None, r, T_dev=B.T, G_dev=B.G)
        self.be.lls_solve(G, kp, k, B.P, True, B.sdd, B.e, B.out, B.etry)
        return DeviceSolve(k, kp, None, None, None, True, True, G, B.out[:3 + k + 3 * k * k], B.etry[:k],
                           hh_dev=B.hh[:ls.k], sc_dev=B.sc)        # sc': entries [:k - 1] valid

    def adopt(self, ls: "DeviceSolve", basis):
        """A speculative solve became the current step: fill its host-side fields from the (now
        updated) host state -- the same values k_lls_next computed on the device."""
        k = ls.k
        self.solves += 1
        self.device_solves += 1
        P, rescale = self._initial_preconditioner(k)
        ls.P = P.copy()
        ls.M = basis.gram_left()
        ls.M_cont = np.diag(np.append(basis.sc[:k - 1], 1.0))

    def finish(self, ls: DeviceSolve, out: np.ndarray):
        """Accept the device solve (host copy ``out`` of ls.out) -> (d, jdd), or None when it needs
        more passes (not SPD, non-finite, or cond(R_Y) > COND_ACCEPT): then ``continue_host``."""
        k = ls.k
        status, jdd = out[0], float(out[1])
        d = out[3:3 + k].copy()
        R = out[3 + k:3 + k + k * k].reshape(k, k).copy()
        Ry = out[3 + k + k * k:3 + k + 2 * k * k].reshape(k, k)
        if status != 0.0 or not (np.isfinite(jdd) and np.all(np.isfinite(d)) and np.all(np.isfinite(R))):
            return None
        cond = _cond_upper(Ry)
        if cond > COND_ACCEPT:
            return None
        self.history.append((k, 1, [cond]))
        if ls.pending:
            self._tentative = (R, d, False)
        else:
            self._settle(R)
        return d, jdd

    def continue_host(self, ls: DeviceSolve, u, basis, r):
        """The device solve needs more passes: continue the CholQR2 / shifted-CholQR passes on the
        host from the first pass's Gram (a pending column has been settled by the trial since: it is
        mapped by ls.M_cont).  -> (d, jdd) in the units of the launch (tentative if it was pending)."""
        self.solves -= 1            # counted again by _passes
        G0 = ls.G.to("cpu").numpy().reshape(ls.kp, ls.kp).copy()
        d, jdd, _ = self._passes(u, basis, ls.k, ls.M_cont, ls.P.copy(), ls.rescale, r, ls.pending, G0=G0,
                                 passes_before=1)
        return d, jdd

    # -- host solve -------------------------------------------------------------------------
    def solve(self, u, basis, r):
        """(d, jdd, R) for min ||-J(u) V d - r|| over the basis' Gram columns.  With a pending column
        d and R are tentative (raw units of that column, messages deferred): see resolve_pending."""
        k = basis.gram_k() if hasattr(basis, "gram_k") else basis.k
        M = basis.gram_left() if hasattr(basis, "gram_left") else None
        pending = getattr(basis, "pending", False)
        P, rescale = self._initial_preconditioner(k)
        if P is not None:
            P = P.copy()
        return self._passes(u, basis, k, M, P, rescale, r, pending)

    def _passes(self, u, basis, k, M, P, rescale, r, pending, G0=None, passes_before=0):
        self.solves += 1
        p0 = self.passes - passes_before
        conds = []
        R = None
        shifted = False                                  # a Gram was numerically singular
        if P is None:
            # classical CholQR2: first pass without preconditioner (T = M, no r column)
            G1 = self._gram(u, basis, k, M, None)[:k, :k]
            try:
                P = _chol_upper(G1)
            except (np.linalg.LinAlgError, ValueError):
                n = self.n_global
                shift = 11.0 * (n * k + k * (k + 1)) * EPS * np.trace(G1)
                P = _chol_upper(G1 + shift * np.eye(k))
                shifted = True
        for it in range(MAX_PASSES):
            if it == 0 and G0 is not None:
                Gp = G0
            else:
                Gp = self._gram(u, basis, k, self._transform(M, P), r)
            if rescale and it == 0:
                # the new column's scale ||J v_new|| from this pass: Y[:, k-1] /= s, P[k-1, k-1] = s
                s2 = Gp[k - 1, k - 1]
                if np.isfinite(s2) and s2 > 0.0:
                    s = np.sqrt(s2)
                    Gp[k - 1, :] /= s
                    Gp[:, k - 1] /= s
                    P[k - 1, k - 1] = s
            try:
                Ry = _chol_upper(Gp[:k, :k])
            except (np.linalg.LinAlgError, ValueError):
                n = self.n_global
                shift = 11.0 * (n * k + k * (k + 1)) * EPS * np.trace(Gp[:k, :k])
                P = _chol_upper(Gp[:k, :k] + shift * np.eye(k)) @ P
                self.fallbacks += 1
                shifted = True
                continue
            conds.append(_cond_upper(Ry))
            if conds[-1] <= COND_ACCEPT or it == MAX_PASSES - 1:
                z = scipy.linalg.solve_triangular(Ry, Gp[:k, k], trans="T", lower=False)
                R = Ry @ P
                break
            P = Ry @ P                                   # one more pass with the improved factor
            self.fallbacks += 1
        if R is None:
            # no pass gave a Cholesky factor (the Gram is singular beyond the shift): minimum-norm
            # solution from the Gram of the plain basis (below)
            d, jdd, R = self._min_norm(u, basis, k, M, r)
            self.history.append((k, self.passes - p0, conds + [np.inf]))
            if pending:
                self._tentative = (R, d, True)           # resolve_pending drops R as a preconditioner
                return d, jdd, R
            self._settle(R)
            self.R_prev = None                           # no usable preconditioner: CholQR2 next time
            return d, jdd, R
        if self.min_norm_if_singular:
            # the dense lstsq branch: scipy.linalg.lstsq (gelsd, cond = eps) returns the minimum-norm
            # solution when J is rank-deficient; J = Q R, so that is R's truncated-SVD solution of
            # R d' = z with the same cut-off (singular values <= eps sigma_max are zero).  Where R
            # comes from a shifted factorisation (a numerically singular Gram) its small singular
            # values are lifted to ~ sqrt(11 n k eps) ||J|| and are no longer below that cut-off:
            # for J with singular values between eps and ~sqrt(n k eps) of sigma_max this branch
            # (like _min_norm, which truncates at the shift) keeps directions gelsd would drop --
            # the two agree for exactly rank-deficient J (tests: rank-1 Jacobians), not in that band.
            U, S, Wt = np.linalg.svd(R)
            keep = S > EPS * S[0]
            if not np.all(keep):
                d = -(Wt[keep].T @ ((U[:, keep].T @ z) / S[keep]))
                jdd = float(np.sum((R @ d) ** 2))
                self.history.append((k, self.passes - p0, conds))
                self._settle(R)
                self.R_prev = None                       # a singular factor does not precondition
                return d, jdd, R
        d = -scipy.linalg.solve_triangular(R, z, lower=False)
        jdd = float(np.sum((R @ d) ** 2))
        self.history.append((k, self.passes - p0, conds))
        if pending:
            self._tentative = (R, d, False)
            return d, jdd, R
        self._settle(R)
        return d, jdd, R

    def _min_norm(self, u, basis, k, M, r):
        """No Cholesky factor at all: d = -w with w the minimum-norm solution of G w = Y^T r, G the
        Gram of Y = J V M (one pass; M maps the stored columns to the reference basis), truncated where
        an eigenvalue of G is below the Gram's rounding bound (the sCholQR3 shift, 11 (n k + k (k+1))
        eps tr G).  R (rank messages, ref:gauss_newton_krylow.py:32-34) is the triangular factor of
        diag(sqrt(lambda)) Q^T, zero on the truncated directions."""
        G = self._gram(u, basis, k, M, r)
        Gk, b = G[:k, :k], G[:k, k]
        lam, Q = np.linalg.eigh(0.5 * (Gk + Gk.T))
        keep = lam > 11.0 * (self.n_global * k + k * (k + 1)) * EPS * max(np.trace(Gk), 0.0)
        w = Q[:, keep] @ ((Q[:, keep].T @ b) / lam[keep])
        d = -w
        R = np.linalg.qr(np.sqrt(np.where(keep, lam, 0.0))[:, None] * Q.T, mode="r")
        jdd = float(w @ (Gk @ w))
        return d, jdd, R

    def _settle(self, R):
        if not self.quiet:
            rank_messages(R)                                         # ref:gauss_newton_krylow.py:32-34
        self.R_prev = self.R_last = R
        self._tentative = None

    def resolve_pending(self, nrm: float) -> np.ndarray:
        """The pending column was settled with norm nrm: R and d in reference units
        (column w -> w / nrm: R[:, -1] / nrm, d[-1] * nrm); prints; returns d."""
        R, d, singular = self._tentative
        R = R.copy()
        d = d.copy()
        R[:, -1] /= nrm
        d[-1] *= nrm
        self._settle(R)
        if singular:
            self.R_prev = None                  # a rank-deficient factor does not precondition the next pass
        return d

    def discard_pending(self):
        """The pending column broke down: the tentative solve is void (R_prev stays)."""
        self._tentative = None
