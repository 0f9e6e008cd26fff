"""CPU oracle for the generalized-Krylov Gauss-Newton hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product package
(``gauss_newton_via_generalized_krylov_subspaces_amd``) never imports it and has
no CPU fallback.

What it is: a NumPy restatement of the reference algorithm
(mariusbaehr/gauss_newton_via_generalized_krylov_subspaces, snapshot 2025-11-28)
written matrix-free for the Bratu operator, so it also runs at grid sizes where
the reference's per-call CSR assembly is too slow.  Every function cites the
reference file:line it restates.  The stencil sums follow scipy's CSR/CSC
row-accumulation order (0 + a1*x1 + a2*x2 + ..., columns ascending) so the
oracle agrees with the reference CSR path to the last bit or two.

Pinning: ``tests/test_oracle_golden.py`` checks this module against
``tests/golden/golden.npz`` / ``golden.json``, which ``tests/golden/make_golden.py``
produced by running the reference itself (OPENBLAS_NUM_THREADS=1, numpy 2.2.6,
scipy 1.15.3).  Third-party arithmetic restated here: scipy 1.15.3
``scipy.sparse.linalg.cg`` (scipy/sparse/linalg/_isolve/iterative.py:305-422) and
LAPACK Householder QR via ``scipy.linalg.qr`` (kept as the real LAPACK call).
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg
import scipy.sparse


# --------------------------------------------------------------------------- exceptions
class GeneralizedKrylowSubspaceBreakdown(Exception):
    """ref:krylow.py:8-9"""


class GeneralizedKrylowSubspaceSpansEntireSpace(Exception):
    """ref:krylow.py:12-13"""


class StepLengthConvergenceError(RuntimeError):
    """ref:armijo_goldstein.py:8-13"""

    def __init__(self, message):
        super().__init__(message)
        self.message = message


class RegressionResult:
    """ref:regression_result.py:4-49 (fields method_name, x, success, nrev, njev, nit)."""

    def __init__(self, method_name, x, success, nrev, njev, nit):
        self.method_name = method_name
        self.x = x
        self.success = success
        self.nrev = nrev
        self.njev = njev
        self.nit = nit

    def __str__(self):
        msg = "converged successfuly to" if self.success else "failed to terminate and stopped at"
        return (f"{self.method_name} {msg} {self.x}. After {self.nit} iterations using "
                f"{self.nrev} evaluations of the residual, ")


# --------------------------------------------------------------------------- Bratu stencil
class BratuStencil:
    """Matrix-free Bratu operator on the N x N interior grid.

    Layout (ref:bratu_pde_problem.py:69-74, meshgrid + flatten("F")): flat index
    ``jx*N + iy`` with jx the x index (slow axis).  Coefficients restate the CSR
    entries of ref:bratu_pde_problem.py:43-67 and :92-96:
      L   = kron(L1, I) + kron(I, L1), times h**-2  -> diag 4*h^-2, neighbours -h^-2
      D_x = kron(diag(-1, +1 super), I), times h**-1 (forward difference along jx)
    """

    def __init__(self, N, alpha, lam, h):
        self.N = int(N)
        self.alpha = alpha
        self.lam = lam
        self.h = h
        hm2 = h ** -2
        hm1 = h ** -1
        self.hm2 = hm2
        self.hm1 = hm1
        self.l_diag = 4.0 * hm2                      # (2+2) * h^-2
        self.l_off = -1.0 * hm2
        self.dx_diag = alpha * (-1.0 * hm1)          # ALPHA * partial_diff_x (matrix scaled first)
        self.dx_up = alpha * (1.0 * hm1)
        self.j_lin_diag = self.l_diag + self.dx_diag  # (L + alpha D_x) diagonal, csr_plus_csr
        self.j_lin_up = self.l_off + self.dx_up       # (L + alpha D_x) entry at column i+N

    # shifted copies with zero Dirichlet ghosts, on the (N, N) [jx, iy] view
    def _nb(self, x):
        X = x.reshape(self.N, self.N)
        z = np.zeros_like(X)
        n_ = z.copy(); n_[1:, :] = X[:-1, :]   # x[i-N]
        s_ = z.copy(); s_[:-1, :] = X[1:, :]   # x[i+N]
        w_ = z.copy(); w_[:, 1:] = X[:, :-1]   # x[i-1]
        e_ = z.copy(); e_[:, :-1] = X[:, 1:]   # x[i+1]
        return X, n_, w_, e_, s_

    def laplace(self, x):
        """L @ x in CSR column order (i-N, i-1, i, i+1, i+N)."""
        X, xn, xw, xe, xs = self._nb(x)
        s = 0.0 + self.l_off * xn
        s = s + self.l_off * xw
        s = s + self.l_diag * X
        s = s + self.l_off * xe
        s = s + self.l_off * xs
        return s.reshape(-1)

    def dx(self, x):
        """(ALPHA * D_x) @ x."""
        X, _, _, _, xs = self._nb(x)
        s = 0.0 + self.dx_diag * X
        s = s + self.dx_up * xs
        return s.reshape(-1)

    def pde_operator(self, u):
        """ref:bratu_pde_problem.py:76-83"""
        if self.lam == 0:
            return self.laplace(u) + self.dx(u)
        return self.laplace(u) + self.dx(u) + self.lam * np.exp(u)

    def diag(self, u):
        """diagonal of (L + alpha D_x + lambda diag e^u), ref:bratu_pde_problem.py:89-96"""
        if self.lam == 0:
            return np.full(self.N * self.N, self.j_lin_diag)
        return self.j_lin_diag + self.lam * np.exp(u)

    def jvp(self, u, v, dg=None):
        """J(u) @ v with J = -(L + alpha D_x + lambda diag e^u), CSR row order."""
        if dg is None:
            dg = self.diag(u)
        X, vn, vw, ve, vs = self._nb(v)
        D = dg.reshape(self.N, self.N)
        s = 0.0 + (-self.l_off) * vn
        s = s + (-self.l_off) * vw
        s = s + (-D) * X
        s = s + (-self.l_off) * ve
        s = s + (-self.j_lin_up) * vs
        return s.reshape(-1)

    def vjp(self, u, w, dg=None):
        """J(u).T @ w, csc_matvec accumulation order (source rows ascending)."""
        if dg is None:
            dg = self.diag(u)
        X, wn, ww, we, ws = self._nb(w)
        D = dg.reshape(self.N, self.N)
        s = 0.0 + (-self.j_lin_up) * wn
        s = s + (-self.l_off) * ww
        s = s + (-D) * X
        s = s + (-self.l_off) * we
        s = s + (-self.l_off) * ws
        return s.reshape(-1)

    def diag_jtj(self, u, dg=None):
        """diag(J^T J) in closed form: sum over the existing neighbours j of J[j, i]^2."""
        if dg is None:
            dg = self.diag(u)
        N = self.N
        D = dg.reshape(N, N)
        out = D * D
        up = np.full((N, N), self.j_lin_up * self.j_lin_up); up[0, :] = 0.0   # J[i-N, i]
        o2 = self.l_off * self.l_off
        west = np.full((N, N), o2); west[:, 0] = 0.0
        east = np.full((N, N), o2); east[:, -1] = 0.0
        south = np.full((N, N), o2); south[-1, :] = 0.0
        return (up + west + out + east + south).reshape(-1)


class BratuJacobian:
    """Matrix-free J(u) with the duck-typed surface the reference consumes:
    ``J @ V`` (n x k), ``J @ v``, ``J.T @ w`` and ``-1 * J`` (ref:gauss_newton.py:113)."""

    def __init__(self, st, u, sign=1.0):
        self.st = st
        self.u = u
        self.sign = sign
        self.shape = (st.N * st.N, st.N * st.N)
        self._dg = st.diag(u)

    def __matmul__(self, V):
        if V.ndim == 1:
            return self.sign * self.st.jvp(self.u, V, self._dg)
        return np.stack([self.__matmul__(V[:, j]) for j in range(V.shape[1])], axis=1)

    def __rmul__(self, s):
        return BratuJacobian(self.st, self.u, self.sign * s)

    __mul__ = __rmul__

    @property
    def T(self):
        parent = self

        class _T:
            def __matmul__(self, w):
                return parent.sign * parent.st.vjp(parent.u, w, parent._dg)

        return _T()

    def diag_ata(self):
        return self.st.diag_jtj(self.u, self._dg)


class BratuPdeProblem:
    """ref:bratu_pde_problem.py:11-99, matrix-free."""

    def __init__(self, grid_nodes, ALPHA, LAMBDA, lower_bound=-3.0, upper_bound=3.0,
                 grid_resolution=None, u=None):
        self.grid_nodes = grid_nodes
        self.ALPHA = ALPHA
        self.LAMBDA = LAMBDA
        self.grid_resolution = ((upper_bound - lower_bound) / grid_nodes
                                if grid_resolution is None else grid_resolution)
        self.N = grid_nodes - 1
        self.stencil = BratuStencil(self.N, ALPHA, LAMBDA, self.grid_resolution)
        lin = np.linspace(lower_bound, upper_bound, grid_nodes + 1)[1:-1]
        self.grid = np.meshgrid(lin, lin)
        f = u if u is not None else (lambda a, b: np.exp(-10 * (a ** 2 + b ** 2)))
        self.u_true = f(*self.grid).flatten("F")

    def pde_operator(self, u):
        return self.stencil.pde_operator(u)

    def make_res(self, y):
        return lambda u: y - self.stencil.pde_operator(u)

    def make_jac(self):
        return lambda u: BratuJacobian(self.stencil, u)

    def make_error(self):
        return lambda u: np.linalg.norm(self.u_true - u)


# --------------------------------------------------------------------------- solver pieces
class KrylovBasis:
    """ref:krylow.py:16-73 (dense basis, CGS1, breakdown atol 1e-8)."""

    def start(self, x0):
        if np.allclose(x0, np.zeros_like(x0)):                     # :31
            raise ValueError("x0 is not allowed to be 0 in the gauss_newton_krylow algorithm")
        nrm = np.linalg.norm(x0)                                   # :36
        self.basis = (x0 / nrm).reshape(-1, 1)                     # :37
        return np.array([nrm])

    def x(self, c):
        return self.basis @ c                                      # :41-42

    def update(self, jac_ev, res_ev):
        if self.basis.shape[0] == self.basis.shape[1]:             # :59-60
            raise GeneralizedKrylowSubspaceSpansEntireSpace
        g = -(jac_ev.T @ res_ev)                                   # :62
        g = g - self.basis @ (self.basis.T @ g)                    # :64
        if np.allclose(g, 0, atol=1e-8, rtol=0):                   # :66
            raise GeneralizedKrylowSubspaceBreakdown("breakdown")
        g = g / np.linalg.norm(g)                                  # :71
        self.basis = np.hstack([self.basis, g.reshape(-1, 1)])     # :72-73


def linear_least_squares(A, y):
    """ref:gauss_newton_krylow.py:16-36 (LAPACK economic QR, rank print, trsv)."""
    q, r = scipy.linalg.qr(A, mode="economic")
    for r_kk in np.diagonal(r):
        if np.isclose(r_kk, 0, atol=1e-8):
            print("A is rank deficient")
    return scipy.linalg.solve_triangular(r, q.T @ y)


def armijo_goldstein(res, x, res_ev, jac_ev, args, d, max_iter=100, initial_step_length=1.0):
    """ref:armijo_goldstein.py:16-72"""
    t = initial_step_length
    prev = np.sum(res_ev ** 2)
    jdd = np.sum((jac_ev @ d) ** 2)
    for it in range(max_iter):
        cur_res = res(x + t * d, *args)
        if prev - np.sum(cur_res ** 2) >= 0.5 * t * jdd:
            return t, cur_res, it + 1
        t /= 2
    raise StepLengthConvergenceError(
        "The armijio_goldstein subroutine reached maximum iteration bound before principle was satisfied! Possible reasons:"
        + "\n- The max iteration count is not big enough to allow for a sufficiently small step size"
        + "\n- Or the descent direction is invalid."
        + f"Norm of descent_direction ={np.linalg.norm(d)}.")


_VERSIONS = ("res_old", "res_new", "jac_old_res_old", "jac_old_res_new")


def gauss_newton_krylow(res, x0, jac, krylow_restart=None, args=(), tol=1e-8, max_iter=100,
                        callback=None, version="res_old", trace=None):
    """ref:gauss_newton_krylow.py:39-145.  ``trace`` (optional list) receives one dict per
    iteration (t, k, halvings) for the parity tests."""
    callback = callback or (lambda **kw: None)
    success = False
    kr = KrylovBasis()
    c = kr.start(x0)                                               # :71
    res_new = res(kr.x(c), *args)                                  # :76
    nfev = 1
    J = jac(x0, *args)                                             # :78 (at x0, not V@c)
    njev = 1
    if krylow_restart is None:
        krylow_restart = max_iter
    it = 0
    for it in range(1, max_iter):                                  # :84
        JV = J @ kr.basis                                          # :86
        r_old = res_new
        d = linear_least_squares(-1 * JV, r_old)                   # :89
        t, res_new, dnfev = armijo_goldstein(
            lambda cc, *a: res(kr.x(cc), *a), c, r_old, JV, args, d)   # :91-93
        nfev += dnfev
        s = np.sum(c ** 2)                                         # :96
        c += t * d                                                 # :98
        callback(x=kr.x(c), nfev=nfev, cg_iter=None)               # :100
        if trace is not None:
            trace.append({"t": t, "k": kr.basis.shape[1], "nfev_delta": dnfev})
        if t ** 2 * np.sum(d ** 2) <= tol ** 2 * s:                # :102
            success = True
            break
        J_old = J
        J = jac(kr.x(c), *args)                                    # :107
        njev += 1
        try:
            if version == "res_old":
                kr.update(J, r_old)
            elif version == "res_new":
                kr.update(J, res_new)
            elif version == "jac_old_res_old":
                kr.update(J_old, r_old)
            elif version == "jac_old_res_new":
                kr.update(J_old, res_new)
            else:
                raise ValueError("Variable version must be in ['res_old','res_new','jac_old_res_old','jac_old_res_new']")
            c = np.append(c, 0)                                    # :124
        except GeneralizedKrylowSubspaceBreakdown:
            print(f"Generalized krylow subspace breakdown at iteration = {it}, basis.shape = {kr.basis.shape}")
        except GeneralizedKrylowSubspaceSpansEntireSpace:
            print("Warning: The genearlized krylow subspace is now identical to the whole parameter "
                  f"space at iteration = {it}")
        if it % krylow_restart == 0:                               # :135
            c = kr.start(kr.x(c))
    if not success:
        print("Warning: The gauss_newton_krylow algorithm reached maximal iteration bound before terminating!")
    return RegressionResult("gauss newton krylow", kr.x(c), success, nfev, njev, it)


# --------------------------------------------------------------------------- CGLS path
def scipy_cg(matvec, b, psolve=None, rtol=1e-5, maxiter=None, callback=None):
    """Restates scipy 1.15.3 scipy.sparse.linalg.cg (iterative.py:305-422) for x0 = 0, atol = 0."""
    bnrm2 = np.linalg.norm(b)
    atol = max(0.0, float(rtol) * float(bnrm2))
    if bnrm2 == 0:
        return b, 0
    n = len(b)
    if maxiter is None:
        maxiter = n * 10
    x = np.zeros_like(b)
    r = b.copy()
    rho_prev = p = None
    for iteration in range(maxiter):
        if np.linalg.norm(r) < atol:
            return x, 0
        z = r if psolve is None else psolve(r)
        rho = np.dot(r, z)
        if iteration > 0:
            p *= rho / rho_prev
            p += z
        else:
            p = np.empty_like(r)
            p[:] = z[:]
        q = matvec(p)
        alpha = rho / np.dot(p, q)
        x += alpha * p
        r -= alpha * q
        rho_prev = rho
        if callback:
            callback(x)
    return x, maxiter


def cg_least_squares(A, y, cg_rtol=1e-4, preconditioner=True):
    """ref:gauss_newton.py:11-60, including the double solve when preconditioner=False
    (:45-48 runs unpreconditioned CG whose result is discarded but whose iterations count)."""
    counter = [0]

    def cb(_x):
        counter[0] += 1

    ata = lambda v: A.T @ (A @ v)                                  # :36
    b = A.T @ y
    if not preconditioner:
        scipy_cg(ata, b, rtol=cg_rtol, callback=cb)                # :45-48
    if hasattr(A, "diag_ata"):
        dinv = 1 / A.diag_ata()                                    # :50-54 closed form
    else:
        dinv = 1 / np.asarray((A.T @ A).diagonal())
    x, _ = scipy_cg(ata, b, psolve=lambda r: dinv * r, rtol=cg_rtol, callback=cb)   # :56-58
    return x, counter[0]


def gauss_newton(res, x0, jac, args=(), tol=1e-8, max_iter=100, step_length_control=armijo_goldstein,
                 callback=None, cg_preconditioner=False, cg_rtol=1e-4):
    """ref:gauss_newton.py:63-138 (sparse/operator Jacobian -> CGLS; dense -> lstsq)."""
    callback = callback or (lambda **kw: None)
    x = x0.copy()
    success = False
    cg_iter = None
    r = res(x, *args)
    nfev = 1
    njev = 0
    it = 0
    for it in range(1, max_iter):
        J = jac(x, *args)
        njev += 1
        if isinstance(J, np.ndarray) and not scipy.sparse.issparse(J):
            d = scipy.linalg.lstsq(-1 * J, r)[0]
        else:
            d, cg_iter = cg_least_squares(-1 * J, r, cg_rtol=cg_rtol, preconditioner=cg_preconditioner)
        t, r, dn = step_length_control(res, x, r, J, args, d)
        nfev += dn
        s = np.sum(x ** 2)
        x += t * d
        callback(x=x, nfev=nfev, cg_iter=cg_iter)
        if t ** 2 * np.sum(d ** 2) <= tol ** 2 * s:
            success = True
            break
    if not success:
        print("Warning: The gauss_newton algorithm reached maximal iteration bound before terminating!")
    return RegressionResult("gauss newton", x, success, nfev, njev, it)


def rosenbrock(p):
    """ref:rosenbrock_problem.py:8-19 -- the sparse Rosenbrock chain with parameter_count = p
    (m = 2(p - 1) residuals); returns (res, jac) as the reference module's functions."""
    def res(x):
        return 2 ** 0.5 * np.concatenate([10 * (x[1:] - x[:-1] ** 2), 1 - x[:-1]])

    def jac(x):
        b1 = 10 * scipy.sparse.eye(p - 1, p, k=1) - 20 * scipy.sparse.diags(x[:-1], shape=(p - 1, p))
        b2 = -scipy.sparse.eye(p - 1, p, k=0)
        return 2 ** 0.5 * scipy.sparse.block_array([[b1], [b2]])

    return res, jac


def bratu_workload(N, alpha=5.0, lam=10.0, seed=42, grid_resolution=None, linear_u0=False):
    """Synthetic Bratu inputs of ref:bratu_pde_test.py:22-36 (and :196-219 when linear_u0)."""
    prob = BratuPdeProblem(N + 1, alpha, lam, grid_resolution=grid_resolution)
    y = prob.pde_operator(prob.u_true)
    if linear_u0:
        u0 = -1 * (prob.make_jac()(np.zeros(N * N)).T @ y)
    else:
        np.random.seed(seed)
        u0 = prob.u_true + 0.1 * np.random.normal(loc=0, scale=1, size=len(prob.u_true))
    return prob, y, u0


def hypot_norm(x):
    return math.sqrt(float(np.dot(x, x)))
