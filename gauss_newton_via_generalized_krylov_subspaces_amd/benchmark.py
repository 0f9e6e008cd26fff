"""Convergence traces of a solver run (ref:benchmark.py:14-55), with the per-iteration error and
loss computed on the GPU.

``benchmark_method(method, res, x0, jac, error, args=(), kwargs={})`` keeps the reference's
signature, its call of ``method(res, x0, jac, args=args, callback=callback, **kwargs)`` and its
return value ``(error_list, loss_list, nfev_list, cg_iter_list)``:
  * error_list / loss_list: ``error(x)`` and ``0.5 * sum(res(x)**2)`` at x0 and at every iterate
    the solver's callback reports (ref:benchmark.py:32-46);
  * nfev_list: residual evaluations per iteration (``reverse_accumulation`` of the callback's
    running count, ref:benchmark.py:14-27);
  * cg_iter_list: the CG iterations of every Gauss-Newton step;
  * a ``StepLengthConvergenceError`` is reported as "Warning: <message>" and ends the run
    (ref:benchmark.py:48-51).

Device traces.  When ``method`` is this package's ``gauss_newton_krylow`` or
``gauss_newton``, ``res`` / ``jac`` come from a ``BratuPdeProblem``'s ``make_res(y)`` /
``make_jac()`` and ``error`` is the same problem's ``make_error()``, the iterate never leaves the
GPU: the solver hands its slab vector to the callback (``callback_format="device"``), the loss is
the solver's own sum of squares of the residual at that point (the accepted Armijo trial's
residual -- the reference re-evaluates ``res`` at the same point) and the error
is one fused pass ``||u_true - x||`` against u_true held on the device.  Per iteration three
scalars reach the host.  Multi-GPU: pass ``kwargs={"comm": ...}`` as for the solvers.  Any other
combination calls the user's functions on host arrays exactly as the reference does.
"""
from __future__ import annotations

import math
from typing import List

import numpy as np

from .armijo_goldstein import StepLengthConvergenceError


def reverse_accumulation(nfev_list: List[int]) -> List[int]:
    """ref:benchmark.py:14-27: running totals -> per-step counts."""
    if not nfev_list:
        return []
    return [nfev_list[0]] + [nfev_list[i] - nfev_list[i - 1] for i in range(1, len(nfev_list))]


def _device_target(method, res, jac, error, args):
    """(problem, y) when the run can keep its traces on the device, else None."""
    from .bratu_pde_problem import BratuError
    from .gauss_newton import gauss_newton
    from .gauss_newton_krylow import gauss_newton_krylow, resolve_bratu
    if args or method not in (gauss_newton, gauss_newton_krylow) or not isinstance(error, BratuError):
        return None
    try:
        bratu = resolve_bratu(res, jac)
    except (TypeError, ValueError):
        return None
    if bratu is None or bratu[0] is not error.problem:
        return None
    return bratu


class _DeviceTraces:
    """u_true and scratch on this rank's slab; error / loss of a slab iterate."""

    def __init__(self, problem, y, kwargs):
        from ._device import BratuDevice
        self.dev = BratuDevice(problem, kwargs.get("comm"), kwargs.get("device"), kwargs.get("_backend"))
        self.be, self.comm = self.dev.backend, self.dev.comm
        self.u_true = self.dev.load(problem.u_true)
        self.y = self.dev.load(y)
        self.tmp = self.dev.vec()
        self.s = self.dev.scalar(3)

    def error(self, x) -> float:
        """||u_true - x|| (ref:bratu_pde_problem.py:98-99) over owned rows: the compensated sum of
        squares as (s, c) pairs merged in rank order (the same value on any rank count)."""
        self.be.vec_axpy(x, -1.0, self.u_true, self.tmp, False)
        self.be.vec_stats(self.tmp, self.s, pairs=True)
        return math.sqrt(self.comm.sum_pairs(self.s, 1)[0])

    def sumsq_residual(self, x) -> float:
        self.be.residual(x, self.y, self.tmp, self.s[0:1])
        return float(self.comm.sum(self.s[0:1])[0])


def benchmark_method(method, res, x0, jac, error, args=(), kwargs={}):
    """Drop-in for ref:benchmark.py:30-55 (see the module docstring)."""
    nfev_list = []
    cg_iter_list = []
    target = _device_target(method, res, jac, error, args)
    if target is not None:
        tr = _DeviceTraces(target[0], target[1], kwargs)
        x0s = tr.dev.load(x0)
        error_list = [tr.error(x0s)]
        loss_list = [0.5 * tr.sumsq_residual(x0s)]

        def callback(x, nfev, cg_iter):
            error_list.append(tr.error(x.x))
            loss_list.append(0.5 * x.sumsq)
            if nfev is not None:
                nfev_list.append(nfev)
            if cg_iter is not None:
                cg_iter_list.append(cg_iter)

        kw = dict(kwargs)
        kw["callback_format"] = "device"
    else:
        def loss(x):
            return 0.5 * np.sum(res(x, *args) ** 2)

        error_list = [error(x0)]
        loss_list = [loss(x0)]

        def callback(x, nfev, cg_iter):
            error_list.append(error(x))
            loss_list.append(loss(x))
            if nfev is not None:
                nfev_list.append(nfev)
            if cg_iter is not None:
                cg_iter_list.append(cg_iter)

        kw = kwargs
    try:
        method(res, x0, jac, args=args, callback=callback, **kw)
    except StepLengthConvergenceError as e:
        print("Warning:", e.message)
    return error_list, loss_list, reverse_accumulation(nfev_list), cg_iter_list
