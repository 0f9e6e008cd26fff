"""Gauss-Newton in generalized Krylov subspaces on MI355X (ref:gauss_newton_krylow.py:39-145).

``gauss_newton_krylow`` keeps the reference's call surface and semantics --
counters (nfev / njev / nit), the ``range(1, max_iter)`` loop bound, the first
Jacobian at x0 but first residual at V @ c, the coordinate-norm convergence
test, the four ``version`` update rules, restart, every printed message and
every exception -- and runs each n-sized operation on the GPU:

  per outer iteration (k basis columns, a Armijo trials)
    1 Gram pass (fp64 MFMA, J V P^-1 on the fly; P = previous R factor, a 2nd pass
      only when the preconditioned factor is not well conditioned) -> LS solve (lls.py)
    a x [basis GEMV + fused residual/||r||^2]   -> Armijo trials
    fused -J^T r + V^T g, CGS update + stats, halo, normalise + ||J v_new|| -> basis update
    (res_old: the first trial's GEMV also yields -J(x)^T r_old and V^T g, from one read of V)

Host <-> device traffic per iteration is O(k^2) doubles (Gram matrices, k
coefficients, a few scalars).  ``GNKSolver`` exposes the same loop one outer
iteration at a time (used by bench.py to time exact steps).

Problems: ``BratuPdeProblem.make_res`` / ``make_jac`` of this package run the
matrix-free Bratu kernels on row slabs (multi-GPU capable); any other ``res`` /
``jac`` callables (the reference's duck typing: ``jac(x)`` returning a scipy sparse
matrix or an ndarray) run through ``generic.HostCallableOps`` -- the user's
functions are evaluated on their NumPy inputs, J and J^T are uploaded as CSR and
every n- and m-sized operation of the loop runs in the HIP library (single GPU).
"""
from __future__ import annotations

from collections.abc import Callable
from typing import Optional

import numpy as np
import torch

from ._device import BratuDevice, DeviceIterate
from .armijo_goldstein import armijo_device
from .bratu_pde_problem import BratuJacobianFunction, BratuResidual
from .krylow import (DeviceKrylovBasis, GeneralizedKrylowSubspaceBreakdown,
                     GeneralizedKrylowSubspaceSpansEntireSpace)
from .lls import CholQR2Solver
from .regression_result import RegressionResult
from .slab import Comm

VERSIONS = ("res_old", "res_new", "jac_old_res_old", "jac_old_res_new")


def _noop(**kwargs):
    return None


def resolve_bratu(res, jac):
    """(problem, y) for the matrix-free Bratu path, None for generic callables."""
    if isinstance(res, BratuResidual) and isinstance(jac, BratuJacobianFunction):
        if res.problem is not jac.problem:
            raise ValueError("res and jac must come from the same BratuPdeProblem")
        return res.problem, res.y
    if isinstance(res, BratuResidual) or isinstance(jac, BratuJacobianFunction):
        raise TypeError("pass both res = BratuPdeProblem.make_res(y) and jac = BratuPdeProblem.make_jac()")
    return None


class BratuOps:
    """Problem side of the GNK loop for the matrix-free Bratu problem: slab vectors on this rank,
    fused residual kernel, the Krylov basis and least-squares solver of this package."""

    jacobian_is_free = True        # J(u) is u itself on the device: no evaluation to schedule
    fuse_trial = True              # the res_old first trial may carry the update products
    speculate = True               # the next step's solve may be enqueued before this one is read

    def __init__(self, problem, y, comm=None, device=None, backend=None):
        self.dev = BratuDevice(problem, comm, device, backend)
        self.be = self.dev.backend
        self.comm = self.dev.comm
        self.n_global = self.dev.slab.n_global
        self.y = self.dev.load(y)
        self._n2 = self.dev.scalar(1)

    def vec(self):
        return self.dev.vec()

    rvec = vec

    def load(self, x0):
        return self.dev.load(x0)

    def residual(self, x, r) -> float:
        self.be.residual(x, self.y, r, self._n2)
        return float(self.comm.sum(self._n2)[0])

    def residual_pack(self, x, r, pack, shared=None):
        """residual partial into pack[0] beside a first trial's device stats (pack[1] = sum w^2,
        pack[2] = max |w|, pack[3:] = V^T g partials): one collective and one host read for all.
        ``shared``: a device buffer that is the same on every rank (the device least-squares
        solve), read in the same round trip -> (rank-combined pack, shared host copy or None)."""
        self.be.residual(x, self.y, r, pack[0:1])
        if shared is None:
            return self.comm.sum_except_max(pack, 2), None
        return self.comm.sum_except_max(pack, 2, shared)

    def residual_read(self, x, r, pack, shared, pinned):
        """``residual_pack`` without waiting: the cross-rank gather and the copy to host are
        enqueued (slab.Comm.read_async) and ``comm.complete`` waits for them, so the host can
        enqueue more work in between; the rank-summed pack stays usable on the device."""
        self.be.residual(x, self.y, r, pack[0:1])
        return self.comm.read_async(pack, shared, pinned)

    def to_host(self, x):
        return self.dev.slab.to_host(x)

    def own(self, x):
        return x[self.dev.slab.own]

    def make_basis(self, kmax):
        return DeviceKrylovBasis(self.dev, kmax)

    def make_lls(self, kmax):
        return CholQR2Solver(self.dev, kmax)

    def on_jacobian(self, u):
        pass


class GNKSolver:
    """One rank of the device GNK loop; ``step()`` runs exactly one outer iteration."""

    # an adopted speculative solve hands its device-formed hh' / sc' to the first trial and to the next
    # speculation instead of uploading the host's copies (two host->device copies per step fewer; the
    # same values: tests/test_gpu_spec_reuse.py runs both ways bit for bit)
    reuse_spec_device = True

    def __init__(self, problem, y, krylow_restart=None, tol=1e-8, max_iter=100, version="res_old",
                 comm: Optional[Comm] = None, device=None, backend=None, callback: Callable = None,
                 callback_format: str = "numpy", ops=None):
        self.ops = ops if ops is not None else BratuOps(problem, y, comm, device, backend)
        self.dev = getattr(self.ops, "dev", None)
        self.be = self.ops.be
        self.comm = self.ops.comm
        self.tol = tol
        self.max_iter = int(max_iter)
        self.version = version
        self.restart = self.max_iter if krylow_restart is None else int(krylow_restart)
        kmax = min(self.restart, max(self.max_iter - 1, 1)) + 1
        kmax = min(kmax, self.ops.n_global)
        self.callback = callback
        self.callback_format = callback_format
        self.basis = self.ops.make_basis(kmax)
        self.lls = self.ops.make_lls(kmax)
        self.xb = [self.ops.vec() for _ in range(3)]
        self.rb = None           # residual buffers: allocated at setup (generic problems learn m there)
        self.trace = []          # per-iteration (t, k, trials) for tests / diagnostics
        # speculative enqueue of the next step's least-squares solve
        self.pipeline = bool(getattr(self.ops, "speculate", False)) and getattr(self.lls, "lsk", 0) > 0
        self._spec = None        # the next step's device solve, enqueued before this step was read
        self._halo_done = False  # the pending column's ghost rows were exchanged for the speculation
        self._par = 0            # device buffer set of the current step's solve (two sets alternate)
        self._pin = None
        self.spec_stats = {"hit": 0, "miss": 0}

    # -- pieces -------------------------------------------------------------------------
    def _residual(self, x, r) -> float:
        return self.ops.residual(x, r)

    def _free_x(self, *busy):
        for i in range(3):
            if i not in busy:
                return i
        raise RuntimeError("no free iterate buffer")

    def _emit(self, xslab, sumsq=None):
        if self.callback is None:
            return
        if self.callback_format == "device":
            x = DeviceIterate(xslab, sumsq, self.ops)
        else:
            x = self.ops.own(xslab) if self.callback_format == "torch" else self.ops.to_host(xslab)
        self.callback(x=x, nfev=self.nfev, cg_iter=None)

    def _pinned(self):
        """Host landing buffer of a step's control scalars (pinned, so the read is enqueued)."""
        if self._pin is None and getattr(self.be, "device", torch.device("cpu")).type == "cuda":
            L = self.lls.lsk
            n = self.comm.world * (4 + self.basis.kmax) + 3 + L + 3 * L * L
            self._pin = torch.empty(n, dtype=torch.float64, pin_memory=True)
        return self._pin

    def _can_speculate(self, it, kk):
        """The next step is a plain continuation of this one when it runs at all: no restart or end
        of the loop after iteration ``it``, and room for one more column in every device buffer."""
        b = self.basis
        return (self.pipeline and it % self.restart != 0 and it < self.max_iter - 1
                and kk + 1 <= min(self.lls.lsk, b.FUSE_KMAX, b.kmax) and kk < self.ops.n_global)

    def _launch_spec(self, ls, rd, x_t, r_t, slot):
        """Enqueue the next step's Gram pass and device solve now, assuming this step
        accepts its first trial, its pending column (if any) does not break down and the res_old
        update appends g = -J(x_t)^T r_old, which the fused trial already wrote into ``slot``:
        the next pass runs at u = x_t with r = r_t."""
        par = self._par ^ 1
        self.basis.halo_slot(slot)
        # k_lls_next reads sc[:k-1] of a pending solve: an adopted speculative solve already holds them
        reuse = self.reuse_spec_device and getattr(ls, "sc_dev", None) is not None and ls.pending
        sc_dev = ls.sc_dev if reuse else self.basis.sc_device(par, ls.k)
        return self.lls.launch_next(x_t, self.basis, r_t, ls, self.comm.device_sum(rd), sc_dev, par)

    def _drop_spec(self):
        if self._spec is not None:
            self._spec = None
            self.spec_stats["miss"] += 1

    # -- loop ---------------------------------------------------------------------------
    def setup(self, x0):
        """ref:gauss_newton_krylow.py:68-82"""
        self.success = False
        self.iter = 0
        self.done = False
        self.uJ = 0                                        # J is evaluated at x0 (:78)
        self.xb[0].copy_(self.ops.load(x0))
        self.c = self.basis.start(self.xb[0])              # :71
        self.e = self.c.copy()                             # stored-unit coordinates (krylow.py)
        self.lls.on_restart()
        xi = self._free_x(self.uJ)
        self.basis.x(self.e, self.xb[xi])
        if self.rb is None:
            self.rb = [self.ops.rvec() for _ in range(2)]
        self.ri = 0
        self.rr = self._residual(self.xb[xi], self.rb[0])  # :76 (at V @ c)
        self.nfev = 1
        self.ops.on_jacobian(self.xb[0])                   # :78 jac(x0)
        self.njev = 1
        if self.max_iter < 2:
            raise UnboundLocalError("local variable 'iter' referenced before assignment")

    def _breakdown_message(self, it):
        print(f"Generalized krylow subspace breakdown at iteration = {it}, basis.shape = {self.basis.shape}")

    def _append_coordinate(self):
        self.c = np.append(self.c, 0)                                     # :124
        self.e = np.append(self.e, 0)

    def _settle_explicit(self):
        """A pending column that no trial will settle (restart, end of the loop): its breakdown test
        and message belong to the iteration that appended it (ref:krylow.py:66, gnk:126-129)."""
        basis = self.basis
        it = basis.pend["it"]
        if basis.resolve_explicit():
            self._breakdown_message(it)
        else:
            self._append_coordinate()

    def _trial_plain(self, e_try, x_t, r_t, r_old, prod):
        """Trial point x_t = V e_try on a settled basis -> (sum r_t^2, raw h or None, product slot)."""
        basis = self.basis
        if not prod:
            basis.x(e_try, x_t)
            return self._residual(x_t, r_t), None, None
        kk = basis.gram_k()
        pack, slot = basis.trial_first(e_try, x_t, r_old)
        host, _ = self.ops.residual_pack(x_t, r_t, pack[:3 + kk])
        return float(host[0]), host[3:3 + kk].copy(), slot

    def _first_trial(self, x_t, r_t, r_old, fuse, it):
        """Least-squares solve (ref:gauss_newton_krylow.py:86-89) and Armijo trial t = 1
        (ref:armijo_goldstein.py:56), enqueued back to back when the solve runs on the device (one
        host read for both).  Settles a pending basis column first -- on its breakdown the solve is
        redone without it -- and, for the fused res_old path, computes the basis-update products at
        the trial point.  A solve the previous step enqueued speculatively for this basis is adopted
        instead of launching one; before waiting for this step's read the next step's solve is
        enqueued the same way when possible.
        Returns (d, jdd, ds, sum r_t^2, raw h or None, product slot); ds = d in stored units."""
        basis, lls = self.basis, self.lls
        u = self.xb[self.uJ]
        spec, self._spec = self._spec, None
        self._par ^= 1
        self._halo_done = False
        while True:
            kk = basis.gram_k()
            pend = basis.pending
            prod = fuse and kk <= basis.FUSE_KMAX
            e_ext = np.append(self.e, np.zeros(kk - len(self.e)))
            sdd = basis.step_scale()
            adopted = spec is not None and pend and spec.k == kk
            if adopted:
                ls = spec
                lls.adopt(ls, basis)
            else:
                ls = lls.launch(u, basis, r_old, e_ext, sdd, par=self._par)
            spec = None
            if not ls.device and not pend:
                ds = sdd * ls.d
                rr, h, slot = self._trial_plain(e_ext + 1.0 * ds, x_t, r_t, r_old, prod)
                return ls.d, ls.jdd, ds, rr, h, slot
            if ls.device:
                # the pack beside the solve's output (lls._LSBuffers.comb): one copy for the step's read
                pk = lls.bufs[self._par].pack if getattr(lls, "bufs", None) else None
                pack, slot = basis.trial_first(None, x_t, r_old if prod else None, coef_dev=ls.e_try,
                                               hh_dev=ls.hh_dev if (adopted and self.reuse_spec_device) else None,
                                               pack=pk)
                rd = self.ops.residual_read(x_t, r_t, pack[:3 + kk], ls.out, self._pinned())
                if prod and self._can_speculate(it, kk):
                    self._spec = self._launch_spec(ls, rd, x_t, r_t, slot)
                host, lsout = self.comm.complete(rd, 2)
                res = lls.finish(ls, lsout)
            else:
                res = (ls.d, ls.jdd)
                pack, slot = basis.trial_first(e_ext + 1.0 * (sdd * ls.d), x_t, r_old if prod else None)
                host, _ = self.ops.residual_pack(x_t, r_t, pack[:3 + kk])
            if pend:
                it_p = basis.pend["it"]
                if basis.resolve(float(host[1]), float(host[2])):
                    # ref:krylow.py:66-69 raised in iteration `it_p`: the basis was not enlarged
                    self._breakdown_message(it_p)
                    lls.discard_pending()
                    self._drop_spec()
                    continue
                self._append_coordinate()                                 # :124 of iteration `it_p`
            if res is None:
                # the device solve needs more passes: finish it on the host, then a new first trial
                self._drop_spec()
                d, jdd = lls.continue_host(ls, u, basis, r_old)
                ds = sdd * d
                if pend:
                    d = lls.resolve_pending(basis.last_norm)
                rr, h, slot = self._trial_plain(self.e + 1.0 * ds, x_t, r_t, r_old, prod)
                return d, jdd, ds, rr, h, slot
            d, jdd = res
            ds = sdd * d
            if pend:
                d = lls.resolve_pending(basis.last_norm)
            # the speculative pass exchanged g's ghost rows
            self._halo_done = self._spec is not None
            return d, jdd, ds, float(host[0]), (host[3:3 + basis.k].copy() if prod else None), slot

    def step(self) -> bool:
        """One pass of ref:gauss_newton_krylow.py:84-136; returns True when the loop has ended."""
        it = self.iter + 1
        basis = self.basis
        r_old = self.rb[self.ri]
        xi = self._free_x(self.uJ)
        rti = 1 - self.ri
        x_t, r_t = self.xb[xi], self.rb[rti]
        # res_old: the update after an accepted first trial is g = -J(x_t)^T r_old, h = V^T g --
        # computed from the same read of V as the trial point itself (speculative)
        fuse = self.ops.fuse_trial and self.version == "res_old"
        d, jdd, ds, rr1, h1, slot1 = self._first_trial(x_t, r_t, r_old, fuse, it)   # :86-89, first trial
        last = {"rr": rr1}
        losses = []                      # every trial's sum r_t^2 (trace: the Armijo comparisons)

        def trial(t):                                                     # res_krylow(c + t d)
            if t == 1.0 and "first" not in last:
                last["first"] = True
                losses.append(rr1)
                return rr1
            basis.x(self.e + t * ds, x_t)
            last["rr"] = self._residual(x_t, r_t)
            losses.append(last["rr"])
            return last["rr"]

        prev_loss = self.rr
        t, ntrial = armijo_device(trial, self.rr, jdd, d)                 # :91-93
        self.nfev += ntrial                                               # :94
        s = np.sum(self.c ** 2)                                           # :96
        self.c += t * d                                                   # :98
        self.e = self.e + t * ds              # the coefficients of the accepted trial point, bit for bit
        self.trace.append({"t": t, "k": basis.k, "trials": ntrial, "prev_loss": prev_loss, "jdd": float(jdd),
                           "losses": losses})
        self._emit(x_t, last["rr"])                                       # :100
        self.iter = it
        self.x_last = xi
        if t ** 2 * np.sum(d ** 2) <= self.tol ** 2 * s:                  # :102-104
            self.success = True
            self.done = True
            self._drop_spec()
            return True
        uJ_old, self.uJ = self.uJ, xi                                     # :106-108
        self.ops.on_jacobian(self.xb[self.uJ])
        self.njev += 1
        u_new = self.xb[self.uJ]
        products = h1 if (h1 is not None and ntrial == 1) else None
        try:
            if self.version == "res_old":
                basis.update(u_new, r_old, it=it, products=products, prod_slot=slot1,
                             halo=not self._halo_done)
            elif self.version == "res_new":
                basis.update(u_new, r_t, it=it)
            elif self.version == "jac_old_res_old":
                basis.update(self.xb[uJ_old], r_old, it=it)
            elif self.version == "jac_old_res_new":
                basis.update(self.xb[uJ_old], r_t, it=it)
            else:
                raise ValueError(
                    "Variable version must be in ['res_old','res_new','jac_old_res_old','jac_old_res_new']")
            if not basis.deferred:
                self._append_coordinate()                                 # :124
                self.lls.on_append()
        except GeneralizedKrylowSubspaceBreakdown:
            self._breakdown_message(it)
        except GeneralizedKrylowSubspaceSpansEntireSpace:
            print("Warning: The genearlized krylow subspace is now identical to the whole parameter space "
                  f"at iteration = {it}")
        self.ri = rti
        self.rr = last["rr"]
        restart = it % self.restart == 0
        if it >= self.max_iter - 1:
            self.done = True
        if basis.pending and self.done and not restart:
            self._settle_explicit()
        if restart:                                                       # :135-136
            xr = self._free_x(self.uJ)
            xstats = None
            if basis.pending and hasattr(basis, "x_settle_start"):
                # the pending column's breakdown test rides on the restart point's GEMV, and the restart
                # point's norm comes back in the same host read
                it_p = basis.pend["it"]
                brk, xstats = basis.x_settle_start(self.e, self.xb[xr])
                if brk:
                    self._breakdown_message(it_p)
                else:
                    self._append_coordinate()
            elif basis.pending and hasattr(basis, "x_settle"):
                it_p = basis.pend["it"]
                if basis.x_settle(self.e, self.xb[xr]):
                    self._breakdown_message(it_p)
                else:
                    self._append_coordinate()
            else:
                if basis.pending:
                    self._settle_explicit()
                basis.x(self.e, self.xb[xr])
            self.c = basis.start(self.xb[xr]) if xstats is None else basis.start(self.xb[xr], stats=xstats)
            self.e = self.c.copy()
            self.lls.on_restart()
        if self._spec is not None:
            # the guess of _launch_spec: first trial accepted, fused products appended as the pending
            # column, no restart / end of the loop
            if (ntrial == 1 and products is not None and not self.done and not restart and basis.pending
                    and basis.gram_k() == self._spec.k):
                self.spec_stats["hit"] += 1
            else:
                self._drop_spec()
        return self.done

    def finish(self, result_format="numpy"):
        """ref:gauss_newton_krylow.py:138-145"""
        if not self.success:
            print("Warning: The gauss_newton_krylow algorithm reached maximal iteration bound before terminating!")
        xi = self._free_x(self.uJ)
        xs = self.basis.x(self.e, self.xb[xi])
        x = self.ops.own(xs).clone() if result_format == "torch" else self.ops.to_host(xs)
        return RegressionResult("gauss newton krylow", x, self.success, self.nfev, self.njev, self.iter)


def gauss_newton_krylow(res, x0, jac, krylow_restart: Optional[int] = None, args: tuple = (), tol: float = 1e-8,
                        max_iter=100, callback: Callable = _noop, version: str = "res_old", *,
                        comm: Optional[Comm] = None, device=None, callback_format: str = "numpy",
                        result_format: str = "numpy", _backend=None) -> RegressionResult:
    """Drop-in for ref:gauss_newton_krylow.py:39-145 (same positional/keyword arguments).

    Extra keyword-only arguments: ``comm`` (a ``slab.Comm``; default: the initialised
    torch.distributed group, else single rank), ``device``, ``callback_format``
    ("numpy": full host vector like the reference; "torch": this rank's device rows),
    ``result_format`` (same choice for ``RegressionResult.x``).
    """
    bratu = resolve_bratu(res, jac)
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
    solver = GNKSolver(problem, y, krylow_restart=krylow_restart, tol=tol, max_iter=max_iter, version=version,
                       comm=comm, device=device, backend=_backend, callback=cb, callback_format=callback_format,
                       ops=ops)
    solver.setup(x0 if not torch.is_tensor(x0) else x0.detach().cpu().numpy())
    while not solver.step():
        pass
    return solver.finish(result_format)
