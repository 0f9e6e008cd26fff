"""CPU test double of the libgnk C-ABI (include/gnk.h), for host-logic tests only.

Implements every backend method of ``_native.HipBackend`` with NumPy on CPU
torch tensors, slab by slab (ghost rows included), so the solver drivers and
the multi-rank slab logic (halo exchange, rank-ordered reductions over gloo) can
be exercised without a GPU.  It is NOT a fallback: the product package never
imports it; tests inject it through the private ``_backend`` argument.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse
import torch

GHOST = 2


class NumpyBackend:
    def __init__(self):
        self.device = torch.device("cpu")
        self.geo = None
        self.pairs = False

    def set_reduce_pairs(self, on):
        """gnk_set_reduce_pairs: compensated results as (s, c) pairs; the double's c is 0."""
        self.pairs = bool(on)

    def _mode(self, pairs, out, plain_len, pair_len, what):
        """As HipBackend._mode: the reduction mode per call, checked against the output's size."""
        need = pair_len if pairs else plain_len
        if out is None or out.numel() < need:
            raise ValueError(f"{what}: output buffer too small for {'pair' if pairs else 'plain'} mode")
        self.pairs = bool(pairs)

    def set_tuning(self, key, value):
        pass

    def scratch_doubles(self):
        return 16 << 20

    def _put(self, out, vals, extra=()):
        """Write compensated results (pairs when enabled), then the plain extras."""
        o = []
        for v in vals:
            o += [float(v), 0.0] if self.pairs else [float(v)]
        o += [float(e) for e in extra]
        for i, v in enumerate(o):
            out[i] = v

    # -- setup -------------------------------------------------------------------------
    def set_bratu(self, N, row0, nrows, h, alpha, lam):
        self.N, self.row0, self.nrows = int(N), int(row0), int(nrows)
        hm2, hm1 = h ** -2, h ** -1
        self.hm2 = -(-1.0 * hm2)
        self.l_off = -1.0 * hm2
        self.l_diag = 4.0 * hm2
        self.dx_diag = alpha * (-1.0 * hm1)
        self.dx_up = alpha * (1.0 * hm1)
        self.j_lin_diag = self.l_diag + self.dx_diag
        self.j_lin_up = self.l_off + self.dx_up
        self.lam = lam

    def slab_len(self):
        return (self.nrows + 2 * GHOST) * self.N

    def empty(self, *shape):
        return torch.empty(*shape, dtype=torch.float64)

    def zeros(self, *shape):
        return torch.zeros(*shape, dtype=torch.float64)

    def upload(self, dst, a):
        a = np.asarray(a, dtype=np.float64).reshape(-1)
        dst.numpy()[:a.size] = a
        return dst

    def to_device(self, a):
        return torch.as_tensor(np.asarray(a, dtype=np.float64)).clone()

    def lls_max_k(self):
        return 32

    def lls_solve(self, G, kp, k, P, rescale, sdd, e, out, e_try):
        """NumPy double of gnk_lls_solve (same layout of out)."""
        import scipy.linalg
        g = G.numpy()[:kp * kp].reshape(kp, kp)[:k + 1, :k + 1].copy()
        p = P.numpy()[:k * k].reshape(k, k).copy()
        s = 1.0
        if rescale:
            s2 = g[k - 1, k - 1]
            if np.isfinite(s2) and s2 > 0.0:
                s = np.sqrt(s2)
                g[k - 1, :] /= s
                g[:, k - 1] /= s
                p[k - 1, k - 1] = s
        o = out.numpy()
        o[:3 + k + 3 * k * k] = np.nan
        try:
            ry = scipy.linalg.cholesky(g[:k, :k], lower=False)
            bad = 0.0
        except (np.linalg.LinAlgError, ValueError):          # not SPD, or NaN (k_lls: t > 0 fails)
            o[0] = 1.0
            return
        z = scipy.linalg.solve_triangular(ry, g[:k, k], trans="T", lower=False)
        R = ry @ p
        d = -scipy.linalg.solve_triangular(R, z, lower=False)
        o[0], o[1], o[2] = bad, float(np.sum((R @ d) ** 2)), s
        o[3:3 + k] = d
        o[3 + k:3 + k + k * k] = R.reshape(-1)
        o[3 + k + k * k:3 + k + 2 * k * k] = ry.reshape(-1)
        o[3 + k + 2 * k * k:3 + k + 3 * k * k] = scipy.linalg.solve_triangular(R, np.eye(k), lower=False).reshape(-1)
        e_try.numpy()[:k] = e.numpy()[:k] + sdd.numpy()[:k] * d

    def lls_next(self, k, pending, out, e_try, pack, sc, kp_next, T, P, sdd, e, hh, scn):
        """NumPy double of gnk_lls_next (the next step's transform, preconditioner, scales)."""
        o, pk = out.numpy(), pack.numpy()
        R = o[3 + k:3 + k + k * k].reshape(k, k)
        rinv = o[3 + k + 2 * k * k:3 + k + 3 * k * k].reshape(k, k)
        nrm = np.sqrt(pk[1]) if pending else 1.0
        s = sc.numpy()[:k].copy()
        dd = np.ones(k)
        if pending:
            s[k - 1] = 1.0 / nrm
            dd[k - 1] = nrm
        h = s * (s * pk[3:3 + k])
        t = np.zeros((kp_next, kp_next))
        t[:k, :k] = (s * dd)[:, None] * rinv
        t[:k, k] = -h
        t[k, k] = t[k + 1, k + 1] = 1.0
        T.numpy()[:kp_next * kp_next] = t.reshape(-1)
        p = np.zeros((k + 1, k + 1))
        p[:k, :k] = R
        if pending:
            p[:k, k - 1] = R[:, k - 1] / nrm
        p[k, k] = 1.0
        P.numpy()[:(k + 1) ** 2] = p.reshape(-1)
        scn.numpy()[:k] = s
        hh.numpy()[:k] = h
        sdd.numpy()[:k + 1] = np.append(s, 1.0)
        e.numpy()[:k + 1] = np.append(e_try.numpy()[:k], 0.0)

    def gram_dim(self, k, with_r):
        return ((k + (1 if with_r else 0) + 15) // 16) * 16

    # -- helpers -----------------------------------------------------------------------
    def _m(self, t):
        return t.numpy().reshape(self.nrows + 2 * GHOST, self.N)

    def _rows(self, lo, hi):
        return slice(lo, hi)

    def _res_rows(self):
        lo, hi = GHOST - 1, GHOST + self.nrows + 1
        if self.row0 == 0:
            lo = GHOST
        if self.row0 + self.nrows >= self.N:
            hi = GHOST + self.nrows
        return lo, hi

    def _diag(self, U):
        if self.lam == 0:
            return np.full_like(U, self.j_lin_diag)
        return self.j_lin_diag + self.lam * np.exp(U)

    def _nb(self, X, lo, hi):
        C = X[lo:hi]
        n_ = X[lo - 1:hi - 1]
        s_ = X[lo + 1:hi + 1]
        w_ = np.zeros_like(C); w_[:, 1:] = C[:, :-1]
        e_ = np.zeros_like(C); e_[:, :-1] = C[:, 1:]
        return n_, w_, C, e_, s_

    def _jvp_block(self, D, vn, vw, vc, ve, vs):
        s = 0.0 + self.hm2 * vn
        s = s + self.hm2 * vw
        s = s + (-D) * vc
        s = s + self.hm2 * ve
        s = s + (-self.j_lin_up) * vs
        return s

    def _vjp_block(self, D, wn, ww, wc, we, ws):
        s = 0.0 + (-self.j_lin_up) * wn
        s = s + self.hm2 * ww
        s = s + (-D) * wc
        s = s + self.hm2 * we
        s = s + self.hm2 * ws
        return s

    # -- operator ----------------------------------------------------------------------
    def jvp(self, u, v, out):
        lo, hi = GHOST, GHOST + self.nrows
        O = self._m(out)
        O[lo:hi] = self._jvp_block(self._diag(self._m(u)[lo:hi]), *self._nb(self._m(v), lo, hi))

    def vjp(self, u, w, out):
        lo, hi = GHOST, GHOST + self.nrows
        O = self._m(out)
        O[lo:hi] = self._vjp_block(self._diag(self._m(u)[lo:hi]), *self._nb(self._m(w), lo, hi))

    def _fwd(self, X, lo, hi):
        xn, xw, xc, xe, xs = self._nb(X, lo, hi)
        l = 0.0 + self.l_off * xn
        l = l + self.l_off * xw
        l = l + self.l_diag * xc
        l = l + self.l_off * xe
        l = l + self.l_off * xs
        dx = 0.0 + self.dx_diag * xc
        dx = dx + self.dx_up * xs
        f = l + dx
        if self.lam != 0:
            f = f + self.lam * np.exp(xc)
        return f

    def forward(self, x, F):
        lo, hi = GHOST, GHOST + self.nrows
        self._m(F)[lo:hi] = self._fwd(self._m(x), lo, hi)

    def residual(self, x, y, r, norm2):
        lo, hi = self._res_rows()
        R = self._m(r)
        R[lo:hi] = self._m(y)[lo:hi] - self._fwd(self._m(x), lo, hi)
        own = R[GHOST:GHOST + self.nrows]
        norm2[0] = float(np.sum(own * own))

    def diag_jtj(self, u, out, reciprocal=False):
        lo, hi = GHOST, GHOST + self.nrows
        D = self._diag(self._m(u)[lo:hi])
        N = self.N
        grow = (self.row0 + np.arange(self.nrows))[:, None]
        iy = np.arange(N)[None, :]
        o2 = self.l_off * self.l_off
        up = np.where(grow > 0, self.j_lin_up * self.j_lin_up, 0.0)
        west = np.where(iy > 0, o2, 0.0)
        east = np.where(iy < N - 1, o2, 0.0)
        south = np.where(grow < N - 1, o2, 0.0)
        v = (((up + west) + D * D) + east) + south
        self._m(out)[lo:hi] = 1.0 / v if reciprocal else v

    def jdiag(self, u, d):
        lo, hi = self._res_rows()
        self._m(d)[lo:hi] = self._diag(self._m(u)[lo:hi])

    # -- basis -------------------------------------------------------------------------
    def gemv(self, V, k, c, x):
        Vn = V.numpy()[:k]
        x.numpy()[:] = np.asarray(c.numpy()[:k]) @ Vn

    # -- flat vectors (generic problems) --------------------------------------------------
    def flat_gemv(self, V, k, c, x):
        x.numpy()[:] = np.asarray(c.numpy()[:k]) @ V.numpy()[:k]

    def flat_gemv_t(self, V, k, g, h):
        h.numpy()[:k] = V.numpy()[:k] @ g.numpy()

    def flat_cgs_update(self, V, k, h, g, stats):
        G = g.numpy()
        G -= h.numpy()[:k] @ V.numpy()[:k]
        stats[0] = float(np.sum(G * G))
        stats[1] = float(np.max(np.abs(G)))

    def flat_stats(self, x, stats, pairs=False):
        self._mode(pairs, stats, 2, 3, 'flat_stats')
        o = x.numpy()
        stats[0] = float(np.sum(o * o))
        stats[1] = float(np.max(np.abs(o)))

    def flat_dot(self, a, b, out, pairs=False):
        self._mode(pairs, out, 1, 2, 'flat_dot')
        out[0] = float(np.dot(a.numpy(), b.numpy()))

    def flat_div(self, src, denom, dst):
        dst.numpy()[:] = src.numpy() / denom

    def flat_axpy(self, x, alpha, d, out):
        out.numpy()[:] = x.numpy() + alpha * d.numpy()

    def flat_cg_update_xr(self, alpha, p, q, x, r, dinv, z, out, pairs=False):
        self._mode(pairs, out, 2, 4, 'flat_cg_update_xr')
        X, R = x.numpy(), r.numpy()
        X[:] = X + alpha * p.numpy()
        R[:] = R - alpha * q.numpy()
        Z = R if dinv is None else 0.0 + dinv.numpy() * R
        if dinv is not None:
            z.numpy()[:] = Z
        out[0] = float(np.dot(R, R))
        out[1] = float(np.dot(R, Z))

    def flat_cg_update_p(self, beta, first, z, p):
        P = p.numpy()
        P[:] = z.numpy() if first else P * beta + z.numpy()

    def csr_spmv(self, nrows, indptr, indices, data, x, y, negate=False, reciprocal=False):
        A = scipy.sparse.csr_array((data.numpy(), indices.numpy(), indptr.numpy()),
                                   shape=(int(nrows), x.numel()))
        v = A @ x.numpy()
        y.numpy()[:] = 1.0 / v if reciprocal else (-v if negate else v)

    def flat_gram(self, W, k, rinv, r, m, G):
        kp = self.gram_dim(k, r is not None)
        Wa = np.zeros((int(m), kp))
        Wa[:, :k] = W.numpy()[:k].T
        if r is not None:
            Wa[:, k] = r.numpy()
        if rinv is not None:
            Wa = Wa @ rinv.numpy().reshape(kp, kp)
        G.numpy()[:] = (Wa.T @ Wa).reshape(-1)

    def gemv_vjp_gemv_t(self, V, k, c, r, x, g, h):
        self.gemv(V, k, c, x)
        self.vjp_gemv_t(x, r, V, k, g, h)

    def gemv_pending(self, V, k, c, hh, x, stats):
        Vn = V.numpy()
        W = Vn[k]
        W[:] = W - np.asarray(hh.numpy()[:k]) @ Vn[:k]
        x.numpy()[:] = np.asarray(c.numpy()[:k + 1]) @ Vn[:k + 1]
        o = W[GHOST * self.N:(GHOST + self.nrows) * self.N]
        stats[0] = float(np.sum(o * o))
        stats[1] = float(np.max(np.abs(o))) if not np.isnan(o).any() else float("nan")

    def gemv_vjp_gemv_t_pending(self, V, k, c, hh, r, x, g, h, stats):
        self.gemv_pending(V, k, c, hh, x, stats)
        self.vjp_gemv_t(x, r, V, k + 1, g, h)

    def vjp_gemv_t(self, u, r, V, k, g, h):
        lo, hi = GHOST, GHOST + self.nrows
        G = self._m(g)
        G[lo:hi] = -self._vjp_block(self._diag(self._m(u)[lo:hi]), *self._nb(self._m(r), lo, hi))
        if k > 0:
            own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
            h.numpy()[:k] = V.numpy()[:k, own] @ g.numpy()[own]

    def cgs_update(self, V, k, h, g, stats):
        own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        gv = g.numpy()
        gv[own] = gv[own] - h.numpy()[:k] @ V.numpy()[:k, own]
        o = gv[own]
        stats[0] = float(np.sum(o * o))
        stats[1] = float(np.max(np.abs(o))) if not np.isnan(o).any() else float("nan")

    def vec_stats(self, x, stats, pairs=False):
        self._mode(pairs, stats, 2, 3, 'vec_stats')
        own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        o = x.numpy()[own]
        self._put(stats, [np.sum(o * o)], [np.max(np.abs(o))])

    def vec_div(self, src, denom, dst, full_slab):
        sl = slice(None) if full_slab else slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        dst.numpy()[sl] = src.numpy()[sl] / denom

    def normalize_jnorm(self, u, g, denom, v, jn2):
        assert g.data_ptr() != v.data_ptr()
        v.numpy()[:] = g.numpy() / denom
        lo, hi = GHOST, GHOST + self.nrows
        jg = self._jvp_block(self._diag(self._m(u)[lo:hi]), *self._nb(self._m(g), lo, hi))
        jn2[0] = float(np.sum(jg * jg))

    def vec_axpy(self, x, alpha, d, out, full_slab):
        sl = slice(None) if full_slab else slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        out.numpy()[sl] = x.numpy()[sl] + alpha * d.numpy()[sl]

    def gram(self, u, V, k, rinv, r, G):
        lo, hi = GHOST, GHOST + self.nrows
        D = self._diag(self._m(u)[lo:hi])
        cols = []
        for j in range(k):
            Vj = V[j].numpy().reshape(self.nrows + 2 * GHOST, self.N)
            cols.append(self._jvp_block(D, *self._nb(Vj, lo, hi)).reshape(-1))
        if r is not None:
            cols.append(self._m(r)[lo:hi].reshape(-1).copy())
        kp = self.gram_dim(k, r is not None)
        W = np.zeros((len(cols[0]), kp))
        W[:, :len(cols)] = np.stack(cols, axis=1)
        if rinv is not None:
            W = W @ rinv.numpy().reshape(kp, kp)
        G.numpy()[:kp * kp] = (W.T @ W).reshape(-1)

    # -- CG ------------------------------------------------------------------------------
    def cg_matvec(self, d, p, q, pq, pairs=False):
        self._mode(pairs, pq, 1, 2, 'cg_matvec')
        # t = J p on owned +-1 rows (inside the domain), then q = J^T t
        lo, hi = GHOST, GHOST + self.nrows
        P = self._m(p)
        Dm = self._m(d)
        T = np.zeros_like(P)
        tlo = max(lo - 1, GHOST - (self.row0 - 0) if self.row0 == 0 else lo - 1)
        tlo = GHOST if self.row0 == 0 else lo - 1
        thi = GHOST + self.nrows if self.row0 + self.nrows >= self.N else hi + 1
        T[tlo:thi] = self._jvp_block(Dm[tlo:thi], *self._nb(P, tlo, thi))
        Q = self._m(q)
        Q[lo:hi] = self._vjp_block(Dm[lo:hi], *self._nb(T, lo, hi))
        own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        self._put(pq, [np.dot(p.numpy()[own], q.numpy()[own])])

    def cg_step_matvec(self, d, z, p_in, p_out, q, beta, first, x, xalpha, pq, pairs=False):
        self._mode(pairs, pq, 1, 2, 'cg_step_matvec')
        # p_out on every slab row (owned + ghost, as the kernel's boundary ranges), lagged x update
        own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        pi, pv, zv = p_in.numpy(), p_out.numpy(), z.numpy()
        pv[:] = zv if first else pi * beta + zv
        if x is not None:
            xv = x.numpy()
            xv[own] = xv[own] + xalpha * pi[own]
        self.cg_matvec(d, p_out, q, pq)

    def cg_step_matvec_dev(self, d, z, p_in, p_out, q, first, x, state, pq):
        st = state.numpy()
        self.cg_step_matvec(d, z, p_in, p_out, q, float(st[0]), first, x, float(st[1]), pq, pairs=True)

    def cg_update_xr_dev(self, state, p, q, x, r, dinv, z, out):
        self.cg_update_xr(float(state.numpy()[2]), p, q, x, r, dinv, z, out, pairs=True)

    def cg_scalars(self, parts, world, stage, state):
        """gnk_cg_scalars: the ranks' pairs merged as slab.Comm.merge_pairs, the scipy-cg coefficients."""
        from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
        st = state.numpy()
        P = parts.numpy().reshape(world, -1)
        if stage == 1:
            pq = float(Comm.merge_pairs(P[:, :2])[0])
            st[6] = pq
            st[2] = st[3] / pq
            return
        rr, rz = (float(v) for v in Comm.merge_pairs(P[:, :4]))
        st[5] = rr
        if stage == 0:
            st[0] = st[1] = st[2] = st[4] = 0.0
            st[3] = rz
            return
        st[4] = st[3]
        st[3] = rz
        st[0] = rz / st[4]
        st[1] = st[2]

    def cg_update_xr(self, alpha, p, q, x, r, dinv, z, out, pairs=False):
        self._mode(pairs, out, 2, 4, 'cg_update_xr')
        own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        xv, rv = (x.numpy() if x is not None else None), r.numpy()
        if xv is not None:
            xv[own] = xv[own] + alpha * p.numpy()[own]
        rv[own] = rv[own] - alpha * q.numpy()[own]
        if dinv is not None:
            z.numpy()[own] = 0.0 + dinv.numpy()[own] * rv[own]
            zz = z.numpy()[own]
        else:
            zz = rv[own]
        self._put(out, [np.dot(rv[own], rv[own]), np.dot(rv[own], zz)])

    def cg_sr_update(self, alpha, beta, first, w, p, s, x, r, dinv, u, out):
        own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        P, S, X, R, U, W = p.numpy(), s.numpy(), x.numpy(), r.numpy(), u.numpy(), w.numpy()
        P[own] = U[own] if first else U[own] + beta * P[own]
        S[own] = W[own] if first else W[own] + beta * S[own]
        X[own] = X[own] + alpha * P[own]
        R[own] = R[own] - alpha * S[own]
        U[own] = 0.0 + dinv.numpy()[own] * R[own] if dinv is not None else R[own]
        out[0] = float(np.dot(R[own], U[own]))
        out[1] = float(np.dot(R[own], R[own]))

    def cg_update_p(self, beta, first, z, p):
        own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        if first:
            p.numpy()[own] = z.numpy()[own]
        else:
            p.numpy()[own] = p.numpy()[own] * beta + z.numpy()[own]
