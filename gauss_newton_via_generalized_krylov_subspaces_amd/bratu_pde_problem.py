"""Bratu PDE problem, matrix-free on the GPU.

Mirrors the constructor and methods of ``BratuPdeProblem``
(ref:bratu_pde_problem.py:11-99): ``pde_operator``, ``make_res``, ``make_jac``,
``make_error``, ``u_true``, ``grid``.  The difference is what ``make_res`` and
``make_jac`` return: the reference returns NumPy closures and per-call CSR
matrices; here they return problem-aware callables that the device solvers in
this package recognise and execute with the HIP stencils of libgnk.so (no
Jacobian is ever assembled).  Called directly on NumPy arrays they still behave
like the reference's closures (the evaluation runs on the GPU and returns NumPy),
so user callbacks such as ``benchmark_method``'s ``loss(x)`` keep working.

The reference's CSR attributes (``laplace1d``, ``laplace2d``, ``partial_diff_x``)
are provided lazily for compatibility; no solver path touches them.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import torch


def default_u(x1, x2):
    """ref:bratu_pde_problem.py:7-8"""
    return np.exp(-10 * (x1 ** 2 + x2 ** 2))


class BratuPdeProblem:
    """n = p = (grid_nodes - 1)**2 unknowns on the interior of [lb, ub]^2."""

    def __init__(self, grid_nodes: int, ALPHA: float, LAMBDA: float, lower_bound: float = -3.0,
                 upper_bound: float = 3.0, grid_resolution: Optional[float] = None,
                 u: Callable = default_u, device=None):
        self.grid_nodes = int(grid_nodes)
        self.ALPHA = ALPHA
        self.LAMBDA = LAMBDA
        self.lower_bound = lower_bound
        self.upper_bound = upper_bound
        if grid_resolution is None:
            self.grid_resolution = (upper_bound - lower_bound) / grid_nodes
        else:
            self.grid_resolution = grid_resolution
        self.u = u
        self.N = self.grid_nodes - 1
        self.device = device
        self._grid = None
        self._u_true = None
        self._eval = None

    # -- host-side reference data (lazy: 8.6 GB at 32768^2) ------------------------
    @property
    def grid(self):
        if self._grid is None:
            lin = np.linspace(self.lower_bound, self.upper_bound, self.grid_nodes + 1)[1:-1]
            self._grid = np.meshgrid(lin, lin)
        return self._grid

    @property
    def u_true(self) -> np.ndarray:
        """ref:bratu_pde_problem.py:74 (Fortran-order flatten: flat index jx*N + iy)."""
        if self._u_true is None:
            lin = np.linspace(self.lower_bound, self.upper_bound, self.grid_nodes + 1)[1:-1]
            if self.u is default_u:
                # exp(-10(x^2 + y^2)) evaluated on the transposed meshgrid == flatten("F")
                xx = lin[:, None]
                yy = lin[None, :]
                self._u_true = np.exp(-10 * (xx ** 2 + yy ** 2)).reshape(-1)
            else:
                self._u_true = self.u(*self.grid).flatten("F")
        return self._u_true

    # -- compatibility CSR views (never used by the solvers) ---------------------------
    @property
    def laplace1d(self):
        import scipy.sparse
        g = self.grid_nodes
        return scipy.sparse.diags_array((-np.ones(g - 2), 2 * np.ones(g - 1), -np.ones(g - 2)), offsets=(-1, 0, 1))

    @property
    def laplace2d(self):
        import scipy.sparse
        eye = scipy.sparse.eye(self.N)
        L = scipy.sparse.kron(self.laplace1d, eye) + scipy.sparse.kron(eye, self.laplace1d)
        return L * self.grid_resolution ** -2

    @property
    def partial_diff_x(self):
        import scipy.sparse
        g = self.grid_nodes
        D = scipy.sparse.kron(scipy.sparse.diags_array((-np.ones(g - 1), np.ones(g - 2)), offsets=(0, 1)),
                              scipy.sparse.eye(g - 1))
        return D * self.grid_resolution ** -1

    # -- device evaluation ------------------------------------------------------------
    def _evaluator(self):
        if self._eval is None:
            from ._device import SingleRankOperator
            self._eval = SingleRankOperator(self, self.device)
        return self._eval

    def pde_operator(self, u):
        """F(u) = L u + ALPHA D_x u + LAMBDA exp(u)  (ref:bratu_pde_problem.py:76-83)."""
        return self._evaluator().forward(u)

    def make_res(self, y):
        """res(u) = y - F(u)  (ref:bratu_pde_problem.py:85-86)."""
        return BratuResidual(self, y)

    def make_jac(self):
        """u -> J(u) = -(L + ALPHA D_x + LAMBDA diag e^u), matrix-free (ref:bratu_pde_problem.py:88-96)."""
        return BratuJacobianFunction(self)

    def make_error(self):
        """u -> ||u_true - u|| (ref:bratu_pde_problem.py:98-99); recognised by ``benchmark_method``."""
        return BratuError(self)


class BratuError:
    """error(u) = ||u_true - u||; ``benchmark.benchmark_method`` evaluates it on the device."""

    def __init__(self, problem: BratuPdeProblem):
        self.problem = problem

    def __call__(self, u):
        return np.linalg.norm(self.problem.u_true - _host(u))


def _host(a):
    if torch.is_tensor(a):
        return a.detach().to("cpu").numpy()
    return np.asarray(a)


class BratuResidual:
    """res(u) = y - F(u); recognised by the device solvers."""

    def __init__(self, problem: BratuPdeProblem, y):
        self.problem = problem
        self.y = y

    def __call__(self, u, *args):
        if args:
            raise TypeError("Bratu residual takes no extra args (ref:bratu_pde_problem.py:86)")
        return _host(self.y) - self.problem._evaluator().forward(u)


class BratuJacobianFunction:
    """jac(u) -> BratuJacobian (matrix-free); recognised by the device solvers."""

    def __init__(self, problem: BratuPdeProblem):
        self.problem = problem

    def __call__(self, u, *args):
        if args:
            raise TypeError("Bratu Jacobian takes no extra args (ref:bratu_pde_problem.py:92)")
        return BratuJacobian(self.problem, u)


class BratuJacobian:
    """Matrix-free J(u) with the duck-typed surface the reference consumes
    (``J @ v``, ``J @ V``, ``J.T @ w``, ``-1 * J``), evaluated on the GPU."""

    def __init__(self, problem: BratuPdeProblem, u, sign: float = 1.0):
        self.problem = problem
        self.u = u
        self.sign = sign
        n = problem.N * problem.N
        self.shape = (n, n)

    def __rmul__(self, s):
        return BratuJacobian(self.problem, self.u, self.sign * float(s))

    __mul__ = __rmul__

    def __neg__(self):
        return BratuJacobian(self.problem, self.u, -self.sign)

    def __matmul__(self, V):
        ev = self.problem._evaluator()
        V = _host(V)
        if V.ndim == 1:
            return self.sign * ev.jvp(self.u, V)
        return np.stack([self.sign * ev.jvp(self.u, V[:, j]) for j in range(V.shape[1])], axis=1)

    @property
    def T(self):
        parent = self

        class _Transposed:
            shape = parent.shape

            def __matmul__(self, w):
                return parent.sign * parent.problem._evaluator().vjp(parent.u, _host(w))

        return _Transposed()

    def diagonal_ata(self):
        """diag(J.T @ J) (sign-independent), closed form on the GPU."""
        return self.problem._evaluator().diag_jtj(self.u)
