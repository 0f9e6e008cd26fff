"""Classical Gauss-Newton with the CGLS inner solve on MI355X (ref:gauss_newton.py:11-138).

Problems: the matrix-free Bratu problem of this package (``BratuGNOps``: slab vectors, fused
stencils, multi-GPU) or any ``res`` / ``jac`` callables (``generic.HostCallableOps``: J uploaded as
CSR per iteration, J v / J^T w / the Jacobi vector in ``gnk_csr_spmv``, flat vector kernels).
Dense-ndarray Jacobians take the reference's ``scipy.linalg.lstsq`` branch (ref:gauss_newton.py:
115-116): the least-squares step is a preconditioned CholeskyQR over the identity basis
on the device (``generic.HostCallableOps.dense_lstsq``, at most 63 parameters).

``cg_least_squares`` restates scipy 1.15.3 ``scipy.sparse.linalg.cg``
(iterative.py:305-422: x0 = 0, atol = rtol * ||b||, strict ``<`` test before
each iteration, ``maxiter = 10 n``) on the normal equations A^T A x = A^T y with
A = -J(u), including the reference's quirk of running an unpreconditioned CG
first when ``preconditioner=False`` (ref:gauss_newton.py:45-48) whose
iterations are counted but whose result is discarded.

Per CG iteration on the GPU: one fused 13-point J^T J p stencil with p . q in
the epilogue (gnk_cg_normal_matvec), one fused x/r/z update with r.r and r.z,
one p update -- 112 n bytes of algorithmic traffic -- and two scalar syncs.
``cg_rtol`` is exposed (the reference hard-codes 1e-4, which stays the default).
"""
from __future__ import annotations

import math
import os
from collections.abc import Callable
from typing import Optional

import numpy as np
import torch

from ._device import BratuDevice, DeviceIterate
from .armijo_goldstein import armijo_device
from .gauss_newton_krylow import _noop, resolve_bratu
from .regression_result import RegressionResult
from .slab import Comm


class BratuGNOps:
    """Problem side of GN / CGLS for the matrix-free Bratu problem (slab vectors on this rank):
    the fused 13-point J^T J p stencil, the closed-form diag(J^T J), halos of p.

    The CG scalars (p.q, r.r, r.z) and the squared norms are compensated (Dot2) sums on the device;
    this rank's context returns them as unevaluated (s, c) pairs (``pairs=True`` per call) and the ranks'
    pairs are merged with TwoSum in rank order (slab.Comm.sum_pairs) before rounding, so a multi-rank
    CG runs on the same exactly rounded scalars as a single rank (ref:gauss_newton.py:11-60)."""

    jacobian_is_free = True

    def __init__(self, problem, y=None, comm=None, device=None, backend=None):
        self.dev = BratuDevice(problem, comm, device, backend)
        self.be = self.dev.backend
        self.comm = self.dev.comm
        self.n_global = self.dev.slab.n_global
        self.y = None if y is None else self.dev.load(y)
        self._n1 = self.dev.scalar(1)              # residual sum of squares (plain reduction)
        self._s1 = self.dev.scalar(2)              # one compensated pair
        self._s2 = self.dev.scalar(4)              # two compensated pairs
        self._st = self.dev.scalar(3)              # vec_stats: (s, c, max |x|)
        self.dvec = self.dev.vec()
        self._jd = None

    def vec(self):
        return self.dev.vec()

    rvec = vec

    def scalar3(self):
        return self.dev.scalar(4)                  # [r.u, r.r] (plain) + the (s, c) pair of u.w

    def load(self, x0):
        return self.dev.load(x0)

    def residual(self, x, r) -> float:
        self.be.residual(x, self.y, r, self._n1)
        return float(self.comm.sum(self._n1)[0])

    def to_host(self, x):
        return self.dev.slab.to_host(x)

    def own(self, x):
        return x[self.dev.slab.own]

    def on_jacobian(self, u):
        pass

    def jvp_sumsq(self, u, d) -> float:
        if self._jd is None:
            self._jd = self.dev.vec()
        self.be.jvp(u, d, self._jd)                                  # jac_ev @ d (ref:armijo_goldstein.py:50)
        return self.sumsq(self._jd)

    def axpy(self, x, t, d, out):
        self.be.vec_axpy(x, t, d, out, True)                         # x + t d (whole slab)

    def sumsq(self, v) -> float:
        self.be.vec_stats(v, self._st, pairs=True)
        return float(self.comm.sum_pairs(self._st, 1)[0])

    # CG pieces
    def cg_rhs(self, u, y, b):
        self.be.vjp_gemv_t(u, y, None, 0, b, None)                   # b = A.T @ y = -(J.T y)

    def cg_prepare(self, u):
        self.be.jdiag(u, self.dvec)                                  # J's diagonal, fixed during CG

    def cg_jacobi(self, u, dinv):
        self.be.diag_jtj(u, dinv, reciprocal=True)                   # ref:gauss_newton.py:50-54

    def cg_normal_matvec(self, p, q) -> float:
        sl = self.dev.slab
        self.comm.halo(p, sl.N, sl.nrows)
        self.be.cg_matvec(self.dvec, p, q, self._s1, pairs=True)
        return float(self.comm.sum_pairs(self._s1, 1)[0])

    def cg_update_xr(self, alpha, p, q, x, r, dinv, z):
        self.be.cg_update_xr(alpha, p, q, x, r, dinv, z, self._s2, pairs=True)
        rr, rz = self.comm.sum_pairs(self._s2, 2)
        return float(rr), float(rz)

    def cg_update_p(self, beta, first, z, p):
        self.be.cg_update_p(beta, first, z, p)

    def cg_finish(self, x):
        sl = self.dev.slab
        self.comm.halo(x, sl.N, sl.nrows)

    # fused iteration (N even): direction update + x update (one iteration late) ride on the
    # normal matvec's loads; the halo moves to z (or r), from which every rank forms p itself
    @property
    def cg_fused(self) -> bool:
        return self.dev.slab.N % 2 == 0 and os.environ.get("GNK_CG_FUSED", "1") != "0"

    def cg_halo(self, z):
        sl = self.dev.slab
        self.comm.halo(z, sl.N, sl.nrows)

    def cg_step_matvec(self, z, p_in, p_out, q, beta, first, x, xalpha) -> float:
        self.be.cg_step_matvec(self.dvec, z, p_in, p_out, q, beta, first, x, xalpha, self._s1, pairs=True)
        return float(self.comm.sum_pairs(self._s1, 1)[0])

    def cg_update_rz(self, alpha, q, r, dinv, z):
        self.be.cg_update_xr(alpha, None, q, None, r, dinv, z, self._s2, pairs=True)
        rr, rz = self.comm.sum_pairs(self._s2, 2)
        return float(rr), float(rz)

    def cg_axpy(self, x, alpha, p):
        self.be.vec_axpy(x, alpha, p, x, False)                     # x + alpha p (owned rows)

    # device-side scalars (DeviceCG._cg_fused_dev): the fused iteration's kernels read alpha / beta from a
    # device state that gnk_cg_scalars forms from the ranks' all-gathered pairs -- no host value between
    # the kernels of an iteration, one (lagged) host read of the state per iteration for the stopping test
    cg_device_scalars = True

    def cgd_state(self):
        return self.dev.scalar(8)

    def _cgd_scalars(self, local, stage, st):
        parts = self.comm.gather_device(local)
        self.be.cg_scalars(parts, self.comm.world, stage, st)

    def cgd_update_rz0(self, q, r, dinv, z, st):
        """z = M r and {r.r, rho = r.z} into the state (the alpha = 0 update before the loop)."""
        self.be.cg_update_xr(0.0, None, q, None, r, dinv, z, self._s2, pairs=True)
        self._cgd_scalars(self._s2[:4], 0, st)

    def cgd_iteration(self, z, p_in, p_out, q, first, x, r, dinv, zbuf, st):
        """One fused iteration with the coefficients on the device: direction + lagged x update + normal
        matvec (alpha = rho / p.q), then r -= alpha q, z = M r (r.r, rho, beta), then z's halo."""
        self.be.cg_step_matvec_dev(self.dvec, z, p_in, p_out, q, first, x, st, self._s1)
        self._cgd_scalars(self._s1[:2], 1, st)
        self.be.cg_update_xr_dev(st, None, q, None, r, dinv, zbuf, self._s2)
        self._cgd_scalars(self._s2[:4], 2, st)
        self.cg_halo(z)

    def cgd_read(self, st):
        """Enqueue the state's copy to the host (pinned, event): a handle for ``cgd_wait``."""
        if st.device.type != "cuda":
            return st.detach().clone()
        if getattr(self, "_cgd_pin", None) is None:
            self._cgd_pin = [torch.empty(8, dtype=torch.float64, pin_memory=True) for _ in range(2)]
            self._cgd_i = 0
        self._cgd_i ^= 1
        host = self._cgd_pin[self._cgd_i]
        host.copy_(st, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(st.device))
        return host, ev

    def cgd_wait(self, h) -> np.ndarray:
        self.comm.counters["host_wait"] += 1
        if isinstance(h, torch.Tensor):
            return h.numpy().copy()
        host, ev = h
        ev.synchronize()
        return host.numpy().copy()

    # single-reduction iteration (cg_variant="single_reduction"): the three scalars of one
    # iteration are partial sums in one device buffer, read with one collective
    def cg_sr_update(self, alpha, beta, first, w, p, s, x, r, dinv, u, buf):
        self.be.cg_sr_update(alpha, beta, first, w, p, s, x, r, dinv, u, buf[0:2])

    def cg_sr_matvec(self, u, w, buf):
        """w = A^T A u and u . w (into buf[2:4], a compensated pair): the row-marching kernel
        (first-iteration form, p_out = u) when N is even, else the point-wise one."""
        out = buf[2:4]
        sl = self.dev.slab
        self.comm.halo(u, sl.N, sl.nrows)
        if self.cg_fused:
            if getattr(self, "_sr_p", None) is None:
                self._sr_p = self.dev.vec()
            self.be.cg_step_matvec(self.dvec, u, u, self._sr_p, w, 0.0, True, None, 0.0, out, pairs=True)
        else:
            self.be.cg_matvec(self.dvec, u, w, out, pairs=True)

    def cg_sr_read(self, buf):
        parts = self.comm._gather(buf)                  # per rank [r.u, r.r, s(u.w), c(u.w)]
        s = parts[0, :2].copy()
        for p in range(1, parts.shape[0]):
            s = s + parts[p, :2]                          # rank order, as Comm.sum
        return float(s[0]), float(s[1]), float(self.comm.merge_pairs(parts[:, 2:4])[0])


class DeviceCG:
    """Device state of the CGLS solve (one rank of a Bratu slab, or a generic problem)."""

    def __init__(self, ops):
        if isinstance(ops, BratuDevice):                              # legacy: a BratuDevice
            ops = BratuGNOps(ops.problem, None, ops.comm, backend=ops.backend)
        self.ops = ops
        v = ops.vec
        self.b, self.x, self.r, self.z, self.p, self.q = v(), v(), v(), v(), v(), v()
        self.p2 = v() if getattr(ops, "cg_fused", False) else None   # double-buffered direction
        self.dinv = v()
        self.total_iters = 0
        # device-side CG scalars (ops.cg_device_scalars) and, without a user callback, the lagged host read
        self.device_scalars = True
        self.lag_reads = True
        self.has_callback = False

    def solve(self, u, y, cg_rtol=1e-4, preconditioner=True, callback=None, maxiter=None, variant="scipy"):
        """x = argmin ||y - A x||, A = -J(u); returns (x, cg_iter) like ref:gauss_newton.py:11-60.
        ``maxiter`` (tooling, bench.py) caps each CG run below scipy's 10 n.  ``variant``:
        "scipy" (the reference's recurrence, parity) or "single_reduction" (Chronopoulos-Gear: the
        same Krylov iterates in exact arithmetic, one reduction per iteration instead of two; not
        bit-compatible with scipy, so iteration counts may differ by rounding)."""
        if variant not in ("scipy", "single_reduction"):
            raise ValueError("cg_variant must be 'scipy' or 'single_reduction'")
        self._variant = variant
        self.has_callback = callback is not None
        ops = self.ops
        ops.cg_rhs(u, y, self.b)                                    # b = A.T @ y
        ops.cg_prepare(u)
        count = [0]

        def cb():
            count[0] += 1
            if callback is not None:
                callback(self.x)

        if not preconditioner:
            self._cg(cg_rtol, None, cb, maxiter)                   # ref:gauss_newton.py:45-48
        ops.cg_jacobi(u, self.dinv)                                # ref:gauss_newton.py:50-54
        self._cg(cg_rtol, self.dinv, cb, maxiter)                  # :56-58
        self.total_iters += count[0]
        ops.cg_finish(self.x)
        return self.x, count[0]

    def _cg(self, rtol, dinv, cb, maxiter=None):
        """scipy iterative.py:305-422 with x0 = 0, atol = 0."""
        if getattr(self, "_variant", "scipy") == "single_reduction":
            return self._cg_single_reduction(rtol, dinv, cb, maxiter)
        if self.p2 is not None:
            if getattr(self.ops, "cg_device_scalars", False) and self.device_scalars:
                return self._cg_fused_dev(rtol, dinv, cb, maxiter)
            return self._cg_fused(rtol, dinv, cb, maxiter)
        ops = self.ops
        bnrm2 = math.sqrt(ops.sumsq(self.b))
        atol = max(0.0, float(rtol) * float(bnrm2))
        self.x.zero_()
        if bnrm2 == 0:
            self.x.copy_(self.b)
            return 0
        maxiter = ops.n_global * 10 if maxiter is None else min(int(maxiter), ops.n_global * 10)
        self.r.copy_(self.b)
        self.p.zero_()
        self.q.zero_()
        # z = M r and (r.r, r.z) via the update kernel with alpha = 0 (x, r unchanged)
        rr, rz = ops.cg_update_xr(0.0, self.p, self.q, self.x, self.r, dinv, self.z)
        z = self.z if dinv is not None else self.r
        rho_prev = None
        for iteration in range(maxiter):
            if math.sqrt(rr) < atol:
                return iteration
            rho = rz
            if iteration > 0:
                ops.cg_update_p(rho / rho_prev, False, z, self.p)
            else:
                ops.cg_update_p(0.0, True, z, self.p)
            pq = ops.cg_normal_matvec(self.p, self.q)
            alpha = rho / pq
            rr, rz = ops.cg_update_xr(alpha, self.p, self.q, self.x, self.r, dinv, self.z)
            rho_prev = rho
            cb()
        return maxiter

    def _cg_fused(self, rtol, dinv, cb, maxiter):
        """The same iteration (same roundings, same scalars) in two kernels: p = z + beta p, x += alpha'
        p' (previous iteration's) and q = A^T A p with p.q; then r -= alpha q, z = M r, r.r, r.z.
        The last x update is applied after the loop."""
        ops = self.ops
        bnrm2 = math.sqrt(ops.sumsq(self.b))
        atol = max(0.0, float(rtol) * float(bnrm2))
        self.x.zero_()
        if bnrm2 == 0:
            self.x.copy_(self.b)
            return 0
        maxiter = ops.n_global * 10 if maxiter is None else min(int(maxiter), ops.n_global * 10)
        self.r.copy_(self.b)
        self.p.zero_()
        self.p2.zero_()
        self.q.zero_()
        rr, rz = ops.cg_update_rz(0.0, self.q, self.r, dinv, self.z)
        z = self.z if dinv is not None else self.r
        ops.cg_halo(z)
        p_in, p_out = self.p, self.p2
        rho_prev = alpha_prev = None
        done = maxiter
        for iteration in range(maxiter):
            if math.sqrt(rr) < atol:
                done = iteration
                break
            rho = rz
            if iteration > 0:
                pq = ops.cg_step_matvec(z, p_in, p_out, self.q, rho / rho_prev, False, self.x, alpha_prev)
            else:
                pq = ops.cg_step_matvec(z, p_in, p_out, self.q, 0.0, True, None, 0.0)
            alpha = rho / pq
            rr, rz = ops.cg_update_rz(alpha, self.q, self.r, dinv, self.z)
            ops.cg_halo(z)
            rho_prev, alpha_prev = rho, alpha
            p_in, p_out = p_out, p_in
            cb()
        if alpha_prev is not None:
            ops.cg_axpy(self.x, alpha_prev, p_in)                       # the last x += alpha p
        return done

    def _cg_fused_dev(self, rtol, dinv, cb, maxiter):
        """``_cg_fused`` with its scalar recurrence on the device (gnk_cg_scalars): the same
        IEEE operations on the same values -- the ranks' pairs merged in rank order, alpha = rho / p.q,
        beta = rho / rho_prev -- so the same bits, but no host value between the kernels of an iteration.
        The host reads the state once per iteration for the stopping test (||r|| < atol); without a user
        callback that read is lagged: iteration j + 1 is enqueued before the host waits for iteration j's
        r.r, so the GPU never idles on the read.  If iteration j's r.r stops the loop, the speculative
        iteration's first kernel has already applied x += alpha_j p_j -- exactly the trailing update
        ``_cg_fused`` applies after its loop -- and its r / z updates are dropped with the solve."""
        ops = self.ops
        bnrm2 = math.sqrt(ops.sumsq(self.b))
        atol = max(0.0, float(rtol) * float(bnrm2))
        self.x.zero_()
        if bnrm2 == 0:
            self.x.copy_(self.b)
            return 0
        maxiter = ops.n_global * 10 if maxiter is None else min(int(maxiter), ops.n_global * 10)
        if maxiter <= 0:                               # scipy's loop does not run: x = x0 = 0, no callback
            return maxiter
        if getattr(self, "_st", None) is None:
            self._st = ops.cgd_state()
        st = self._st
        self.r.copy_(self.b)
        self.p.zero_()
        self.p2.zero_()
        self.q.zero_()
        ops.cgd_update_rz0(self.q, self.r, dinv, self.z, st)
        z = self.z if dinv is not None else self.r
        ops.cg_halo(z)
        if math.sqrt(float(ops.cgd_wait(ops.cgd_read(st))[5])) < atol:
            return 0
        P = (self.p, self.p2)
        lag = self.lag_reads and not self.has_callback

        def enqueue(j):
            ops.cgd_iteration(z, P[j % 2], P[(j + 1) % 2], self.q, j == 0, self.x if j > 0 else None,
                              self.r, dinv, self.z, st)

        j = 0
        enqueue(0)
        while True:
            h = ops.cgd_read(st)                       # the state after iteration j
            nxt = j + 1 < maxiter
            if nxt and lag:
                enqueue(j + 1)                         # speculative: runs while the host waits
            sv = ops.cgd_wait(h)
            cb()
            if math.sqrt(float(sv[5])) < atol or not nxt:      # scipy's stop at the next iteration's top,
                if not (nxt and lag):                           # or the iteration cap
                    ops.cg_axpy(self.x, float(sv[2]), P[(j + 1) % 2])    # the last x += alpha p
                return j + 1
            if not lag:
                enqueue(j + 1)
            j += 1

    def _cg_single_reduction(self, rtol, dinv, cb, maxiter):
        """Chronopoulos-Gear PCG (non-parity option): with u = M r, w = A u,
        gamma = r . u, delta = u . w the step and direction coefficients follow from one reduction:
            beta = gamma / gamma_prev,  alpha = gamma / (delta - beta gamma / alpha_prev)
            p = u + beta p,  s = w + beta s (= A p),  x += alpha p,  r -= alpha s,  u = M r
        Stopping and counting as scipy: the loop ends when ||r|| < rtol ||b|| (tested on the residual
        of the last update), each update is one iteration; x0 = 0."""
        ops = self.ops
        if getattr(self, "_sr", None) is None:
            v = ops.vec
            self._sr = (v(), v(), v(), ops.scalar3())          # u, w, s, [r.u, r.r, u.w]
        u, w, sv, buf = self._sr
        bnrm2 = math.sqrt(ops.sumsq(self.b))
        atol = max(0.0, float(rtol) * float(bnrm2))
        self.x.zero_()
        if bnrm2 == 0:
            self.x.copy_(self.b)
            return 0
        maxiter = ops.n_global * 10 if maxiter is None else min(int(maxiter), ops.n_global * 10)
        self.r.copy_(self.b)
        if math.sqrt(ops.sumsq(self.r)) < atol:
            return 0
        # u0 = M r0 (alpha = 0 update: x, r unchanged, p = u, s = w are overwritten below)
        w.zero_()
        ops.cg_sr_update(0.0, 0.0, True, w, self.p, sv, self.x, self.r, dinv, u, buf)
        ops.cg_sr_matvec(u, w, buf)
        gamma, rr, delta = ops.cg_sr_read(buf)
        alpha, beta, first = gamma / delta, 0.0, True
        for iteration in range(maxiter):
            ops.cg_sr_update(alpha, beta, first, w, self.p, sv, self.x, self.r, dinv, u, buf)
            ops.cg_sr_matvec(u, w, buf)
            gamma_new, rr, delta = ops.cg_sr_read(buf)
            cb()
            if math.sqrt(rr) < atol:
                return iteration + 1
            beta = gamma_new / gamma
            alpha_prev = alpha
            alpha = gamma_new / (delta - beta * gamma_new / alpha_prev)
            gamma, first = gamma_new, False
        return maxiter


def cg_least_squares(A, y, x0=None, cg_rtol=1e-4, preconditioner=True):
    """Drop-in for ref:gauss_newton.py:11-60 with A = -jac(u) (a matrix-free BratuJacobian
    scaled by -1) and y a host vector.  Returns (x as numpy, cg_iter)."""
    from .bratu_pde_problem import BratuJacobian
    if x0 is not None:
        raise NotImplementedError("x0 != None is not used by the reference (ref:gauss_newton.py:112-114)")
    if not isinstance(A, BratuJacobian) or A.sign != -1.0:
        raise TypeError("cg_least_squares on MI355X expects A = -1 * jac(u) from BratuPdeProblem.make_jac()")
    ops = BratuGNOps(A.problem, None, Comm(single=True))
    cg = DeviceCG(ops)
    u = ops.load(A.u if not torch.is_tensor(A.u) else A.u.cpu().numpy())
    ys = ops.load(y)
    x, it = cg.solve(u, ys, cg_rtol=cg_rtol, preconditioner=preconditioner)
    return ops.to_host(x), it


class GNSolver:
    """Device Gauss-Newton loop (ref:gauss_newton.py:63-138), one outer iteration per ``step()``."""

    def __init__(self, problem, y, tol=1e-8, max_iter=100, cg_preconditioner=False, cg_rtol=1e-4,
                 comm: Optional[Comm] = None, device=None, backend=None, callback: Callable = None,
                 callback_format="numpy", ops=None, cg_variant="scipy", cg_maxiter=None):
        # cg_maxiter (tooling: bench / full-size tests) caps every CG run below scipy's 10 n
        self.ops = ops if ops is not None else BratuGNOps(problem, y, comm, device, backend)
        self.cg_maxiter = cg_maxiter
        self.dev = getattr(self.ops, "dev", None)
        self.be = self.ops.be
        self.comm = self.ops.comm
        self.tol, self.max_iter = tol, int(max_iter)
        self.cg_pre, self.cg_rtol = cg_preconditioner, cg_rtol
        self.cg_variant = cg_variant
        self.callback, self.callback_format = callback, callback_format
        self.cg = DeviceCG(self.ops)
        self.xb = [self.ops.vec(), self.ops.vec()]
        self.rb = None
        self.trace = []

    def _residual(self, x, r):
        return self.ops.residual(x, r)

    def _dvec(self):
        if getattr(self, "_d", None) is None:
            self._d = self.ops.vec()
        return self._d

    def setup(self, x0):
        self.xi, self.ri = 0, 0
        self.xb[0].copy_(self.ops.load(x0))                          # x = x0.copy() (:95)
        if self.rb is None:
            self.rb = [self.ops.rvec(), self.ops.rvec()]
        self.rr = self._residual(self.xb[0], self.rb[0])             # :100
        self.nfev, self.njev = 1, 0
        self.cg_iter = None
        self.success = False
        self.iter = 0
        self.done = False
        if self.max_iter < 2:
            raise UnboundLocalError("local variable 'iter' referenced before assignment")

    def step(self):
        it = self.iter + 1
        ops = self.ops
        x, r = self.xb[self.xi], self.rb[self.ri]
        ops.on_jacobian(x)                                           # J = jac(x) (:107)
        self.njev += 1                                               # :108
        if getattr(ops, "jacobian_is_dense", None) is not None and ops.jacobian_is_dense(x):
            d = ops.dense_lstsq(x, r, self._dvec())                 # :115-116 (cg_iter keeps its value)
        else:
            d, self.cg_iter = self.cg.solve(x, r, cg_rtol=self.cg_rtol, preconditioner=self.cg_pre,  # :111-114
                                            variant=self.cg_variant, maxiter=self.cg_maxiter)
        jdd = ops.jvp_sumsq(x, d)                                    # sum((J d)^2) (ref:armijo_goldstein.py:50)
        xt, rt = self.xb[1 - self.xi], self.rb[1 - self.ri]
        last = {}

        def trial(t):
            ops.axpy(x, t, d, xt)                                    # x + t d
            last["rr"] = self._residual(xt, rt)
            return last["rr"]

        t, ntrial = armijo_device(trial, self.rr, jdd, d_norm_host(self, d))
        self.nfev += ntrial
        s = ops.sumsq(x)                                             # np.sum(x**2) (:123)
        dd = ops.sumsq(d)
        self.xi, self.ri = 1 - self.xi, 1 - self.ri                  # x += t d (:125) == trial point
        self.rr = last["rr"]
        self.iter = it
        self.trace.append({"t": t, "trials": ntrial, "cg_iter": self.cg_iter})
        if self.callback is not None:
            xs = self.xb[self.xi]
            if self.callback_format == "device":
                xo = DeviceIterate(xs, self.rr, ops)
            else:
                xo = ops.own(xs) if self.callback_format == "torch" else ops.to_host(xs)
            self.callback(x=xo, nfev=self.nfev, cg_iter=self.cg_iter)
        if t ** 2 * dd <= self.tol ** 2 * s:                         # :129-131
            self.success = True
            self.done = True
        elif it >= self.max_iter - 1:
            self.done = True
        return self.done

    def finish(self, result_format="numpy"):
        if not self.success:
            print("Warning: The gauss_newton algorithm reached maximal iteration bound before terminating!")
        xs = self.xb[self.xi]
        x = self.ops.own(xs).clone() if result_format == "torch" else self.ops.to_host(xs)
        return RegressionResult("gauss newton", x, self.success, self.nfev, self.njev, self.iter)


class _DNorm:
    """Lazy ||d|| for the StepLengthConvergenceError message only."""

    def __init__(self, solver, d):
        self.solver, self.d = solver, d

    def __array__(self, dtype=None, copy=None):
        return np.array([math.sqrt(self.solver.ops.sumsq(self.d))])


def d_norm_host(solver, d):
    return _DNorm(solver, d)


def gauss_newton(res, x0, jac, args: tuple = (), tol: float = 1e-8, max_iter=100, step_length_control=None,
                 callback: Callable = _noop, cg_preconditioner: bool = False, *, cg_rtol: float = 1e-4,
                 cg_variant: str = "scipy",
                 comm: Optional[Comm] = None, device=None, callback_format: str = "numpy",
                 result_format: str = "numpy", _backend=None) -> RegressionResult:
    """Drop-in for ref:gauss_newton.py:63-138; ``cg_rtol`` added, and ``cg_variant="single_reduction"``
    (Bratu path) selects the one-reduction CG recurrence (not bit-compatible with scipy)."""
    bratu = resolve_bratu(res, jac)
    if step_length_control is not None:
        raise NotImplementedError("the device solver uses the reference's armijo_goldstein rule")
    cb = None if (callback is None or callback is _noop) else callback
    if bratu is not None:
        if args:
            raise TypeError("<lambda>() takes 1 positional argument but {} were given".format(1 + len(args)))
        problem, y = bratu
        ops = None
    else:
        from .problem import make_generic_ops
        problem, y = None, None
        ops = make_generic_ops(res, jac, x0, args, device=device, backend=_backend)
    if cg_variant != "scipy" and ops is not None:
        raise NotImplementedError("cg_variant='single_reduction' is implemented for the matrix-free Bratu path")
    solver = GNSolver(problem, y, tol=tol, max_iter=max_iter, cg_preconditioner=cg_preconditioner, cg_rtol=cg_rtol,
                      comm=comm, device=device, backend=_backend, callback=cb, callback_format=callback_format,
                      ops=ops, cg_variant=cg_variant)
    solver.setup(x0 if not torch.is_tensor(x0) else x0.detach().cpu().numpy())
    while not solver.step():
        pass
    return solver.finish(result_format)
