"""Matrix-free problems on device tensors: ``Problem(residual, jvp, vjp)``.

The reference's solvers take a residual ``res(x, *args)`` and a Jacobian ``jac(x, *args)`` that they
use only through ``J @ V`` (ref:gauss_newton_krylow.py:86), ``J.T @ r`` (ref:krylow.py:62),
``J @ d`` (ref:armijo_goldstein.py:50) and ``A.T @ (A @ x)`` (ref:gauss_newton.py:36).  A ``Problem``
states exactly that contract on the GPU, so a problem other than Bratu never leaves the device:

  residual(x, *args)   -> r = res(x)       x: (n,) float64 tensor on the solver's device, r: (m,)
  jvp(x, v, *args)     -> J(x) v           (m,)   J = d residual / d x, the reference's ``jac``
  vjp(x, w, *args)     -> J(x)^T w         (n,)
  diag_jtj(x, *args)   -> diag(J(x)^T J(x)) (n,)  optional: the CGLS Jacobi preconditioner
                                                   (ref:gauss_newton.py:50-54); without it the diagonal
                                                   is probed with n JVPs of unit vectors (n <= 65536)

``jvp`` / ``vjp`` default to forward- / reverse-mode derivatives of ``residual`` (torch.func), so
``Problem(residual)`` alone is a complete problem when the residual is written in torch operations.
The callables must not modify their arguments.

``gauss_newton_krylow(prob.make_res(), x0, prob.make_jac())`` (or ``gauss_newton(...)``) then runs:
the user's callables for every residual and Jacobian product, and libgnk for the rest -- the flat
Krylov basis, CGS update and breakdown statistics, the Gram of [J V P^-1 | r] on MFMA (k device JVPs
into the arena, then ``gnk_flat_gram``), the CholeskyQR least-squares solve, the Armijo sums, the
CGLS vector updates and dot products.  Host traffic per outer iteration is O(k^2) doubles, as for
Bratu.  Called directly, ``make_res()`` / ``make_jac()`` behave like the reference's closures (NumPy
in, NumPy out; the Jacobian an operator with ``@`` / ``.T @`` / ``-1 *``), so they also drop into the
reference's own solvers.
"""
from __future__ import annotations

import numpy as np
import torch

from .generic import PROBE_NMAX, HostCallableOps

__all__ = ["Problem", "ProblemResidual", "ProblemJacobianFunction", "ProblemJacobian", "ProblemOps"]


def _auto_jvp(residual):
    def jvp(x, v, *args):
        return torch.func.jvp(lambda z: residual(z, *args), (x,), (v,))[1]
    return jvp


def _auto_vjp(residual):
    def vjp(x, w, *args):
        _, pull = torch.func.vjp(lambda z: residual(z, *args), x)
        return pull(w)[0]
    return vjp


class Problem:
    """A least-squares problem min ||residual(x)||^2 given by device-tensor callables (see module doc)."""

    def __init__(self, residual, jvp=None, vjp=None, *, diag_jtj=None, device=None):
        if not callable(residual):
            raise TypeError("Problem: residual must be callable")
        self.residual = residual
        self.jvp = jvp if jvp is not None else _auto_jvp(residual)
        self.vjp = vjp if vjp is not None else _auto_vjp(residual)
        self.diag_jtj = diag_jtj
        self.device = device
        self.m = None              # learnt from the first residual evaluation

    def _dev(self):
        if self.device is not None:
            return torch.device(self.device)
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    def make_res(self):
        """x -> residual(x): the ``res`` argument of the solvers (ref:gauss_newton_krylow.py:40)."""
        return ProblemResidual(self)

    def make_jac(self):
        """x -> J(x) (an operator): the ``jac`` argument of the solvers (ref:gauss_newton_krylow.py:42)."""
        return ProblemJacobianFunction(self)


def _tensor(a, dev):
    if torch.is_tensor(a):
        return a.detach().to(device=dev, dtype=torch.float64).reshape(-1)
    return torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev).reshape(-1)


def _like(a, t):
    """Return ``t`` in the caller's array type: NumPy in -> NumPy out, tensor in -> tensor out."""
    return t if torch.is_tensor(a) else t.detach().cpu().numpy()


class ProblemResidual:
    """``res(x, *args)`` of a ``Problem``; recognised by the device solvers."""

    def __init__(self, problem: Problem):
        self.problem = problem

    def __call__(self, x, *args):
        p = self.problem
        r = _tensor(p.residual(_tensor(x, p._dev()), *args), p._dev())
        p.m = r.numel()
        return _like(x, r)


class ProblemJacobianFunction:
    """``jac(x, *args)`` of a ``Problem`` -> ``ProblemJacobian``; recognised by the device solvers."""

    def __init__(self, problem: Problem):
        self.problem = problem

    def __call__(self, x, *args):
        return ProblemJacobian(self.problem, _tensor(x, self.problem._dev()), args)


class ProblemJacobian:
    """J(x) as the operator the reference consumes: ``J @ v``, ``J @ V`` ((n, k) columns), ``J.T @ w``,
    ``-J`` / ``s * J`` and ``diagonal_ata()``; NumPy or tensor operands."""

    def __init__(self, problem, x, args=(), sign=1.0, transposed=False):
        self.problem, self.x, self.args, self.sign, self.transposed = problem, x, tuple(args), float(sign), transposed

    @property
    def shape(self):
        p = self.problem
        if p.m is None:
            p.m = _tensor(p.residual(self.x, *self.args), p._dev()).numel()
        n = self.x.numel()
        return (n, p.m) if self.transposed else (p.m, n)

    def __rmul__(self, s):
        return ProblemJacobian(self.problem, self.x, self.args, self.sign * float(s), self.transposed)

    __mul__ = __rmul__

    def __neg__(self):
        return self.__rmul__(-1.0)

    @property
    def T(self):
        return ProblemJacobian(self.problem, self.x, self.args, self.sign, not self.transposed)

    def _apply(self, v):
        p = self.problem
        f = p.vjp if self.transposed else p.jvp
        out = _tensor(f(self.x, v, *self.args), p._dev())
        return out if self.sign == 1.0 else self.sign * out

    def __matmul__(self, V):
        dev = self.problem._dev()
        if torch.is_tensor(V):
            Vt = V.detach().to(device=dev, dtype=torch.float64)
        else:
            Vt = torch.as_tensor(np.asarray(V, dtype=np.float64), device=dev)
        if Vt.ndim == 1:
            return _like(V, self._apply(Vt))
        cols = [self._apply(Vt[:, j].contiguous()) for j in range(Vt.shape[1])]
        return _like(V, torch.stack(cols, dim=1))

    def diagonal_ata(self):
        """diag(J^T J) (sign-independent): ``diag_jtj`` when given, else probed."""
        p = self.problem
        d = torch.empty(self.x.numel(), dtype=torch.float64, device=p._dev())
        _diag_jtj(p, self.x, self.args, d, lambda a, o: o.copy_(torch.dot(a, a)))
        return d.cpu().numpy()


def _diag_jtj(p, x, args, out, sumsq_into):
    """out = diag(J(x)^T J(x)): the Problem's diag_jtj, else sum(col_j^2) over the probed columns
    J e_j (``sumsq_into(col, out[j:j+1])``)."""
    if p.diag_jtj is not None:
        out.copy_(_tensor(p.diag_jtj(x, *args), out.device))
        return
    n = x.numel()
    if n > PROBE_NMAX:
        raise NotImplementedError(f"Problem of {n} unknowns without diag_jtj: gauss_newton's Jacobi preconditioner "
                                  f"(ref:gauss_newton.py:50-54) probes J column by column only up to n = {PROBE_NMAX}")
    e = torch.zeros(n, dtype=torch.float64, device=out.device)
    for j in range(n):
        e[j] = 1.0
        col = _tensor(p.jvp(x, e, *args), out.device)
        sumsq_into(col, out[j:j + 1])
        e[j] = 0.0


class _DeviceJacobian:
    """J at one iterate buffer for the solvers (the interface of generic.DeviceCSR): every product is the
    Problem's own device callable writing into the solver's buffers."""

    def __init__(self, ops, u):
        self.ops, self.u = ops, u
        self.shape = (ops.m, ops.n)

    def _put(self, t, y, negate, what):
        t = _tensor(t, y.device)
        if t.numel() != y.numel():
            raise ValueError(f"Problem.{what} returned {t.numel()} values, expected {y.numel()}")
        y.copy_(t)
        if negate:
            y.neg_()

    def matvec(self, x, y, negate=False):
        p = self.ops.problem
        self._put(p.jvp(self.u, x, *self.ops.args), y, negate, "jvp")

    def rmatvec(self, w, y, negate=False):
        p = self.ops.problem
        self._put(p.vjp(self.u, w, *self.ops.args), y, negate, "vjp")

    def matmat_rows(self, V, k, W):
        for j in range(k):
            self.matvec(V[j], W[j])

    def jacobi(self, ones_m, dinv):
        """dinv = 1 / diag(J^T J) (ref:gauss_newton.py:50-54)."""
        be = self.ops.be
        _diag_jtj(self.ops.problem, self.u, self.ops.args, dinv, lambda a, o: be.flat_dot(a, a, o))
        torch.reciprocal(dinv, out=dinv)


class ProblemOps(HostCallableOps):
    """Problem side of the GNK / GN loops for a device ``Problem``: the user's residual and products run on
    the solver's device tensors (no host copy of any n- or m-sized vector), the rest in libgnk."""

    def __init__(self, problem: Problem, n: int, args=(), device=None, backend=None):
        super().__init__(problem.residual, None, n, args, device=device, backend=backend)
        self.problem = problem
        if problem.device is None:
            problem.device = self.be.device

    def residual(self, x, r) -> float:
        """r = residual(x, *args) on the device; returns sum(r^2) (libgnk reduction)."""
        rv = _tensor(self.problem.residual(x, *self.args), self.be.device)
        if self.m is None:
            self.m = rv.numel()
            self.problem.m = self.m
        if r.numel() == 0:
            r.resize_(rv.numel())
        if rv.numel() != r.numel():
            raise ValueError(f"Problem.residual returned {rv.numel()} values, expected {r.numel()}")
        r.copy_(rv)
        self.be.flat_stats(r, self._st)
        return float(self._st[0].item())

    def on_jacobian(self, u):
        """jac(u): nothing to evaluate up front -- the products take u (ref:gauss_newton_krylow.py:78, :108)."""
        self._dense[u.data_ptr()] = False
        self._J[u.data_ptr()] = _DeviceJacobian(self, u)


def resolve_problem(res, jac):
    """The device Problem behind (res, jac), or None for other callables."""
    if isinstance(res, Problem) and jac is None:
        return res
    if isinstance(res, ProblemResidual) and isinstance(jac, ProblemJacobianFunction):
        if res.problem is not jac.problem:
            raise ValueError("res and jac must come from the same Problem")
        return res.problem
    if isinstance(res, ProblemResidual) or isinstance(jac, ProblemJacobianFunction):
        raise TypeError("pass both res = Problem.make_res() and jac = Problem.make_jac()")
    return None


def make_generic_ops(res, jac, x0, args=(), device=None, backend=None):
    """Problem side for callables that are not the matrix-free Bratu pair: a device ``Problem``
    (ProblemOps) or the reference's NumPy closures (generic.HostCallableOps)."""
    x0h = x0.detach().cpu().numpy() if torch.is_tensor(x0) else np.asarray(x0, dtype=np.float64)
    prob = resolve_problem(res, jac)
    if prob is not None:
        return ProblemOps(prob, x0h.size, args, device=device, backend=backend)
    if jac is None:
        raise TypeError("jac is required unless res is a Problem")
    return HostCallableOps(res, jac, x0h.size, args, device=device, backend=backend)
