"""Generic problems on the device: any ``res`` / ``jac`` callables.

The reference duck-types its problem (ref:gauss_newton_krylow.py:39-49): ``res(x, *args)``
returns the residual vector and ``jac(x, *args)`` anything supporting ``J @ V``, ``J @ v`` and
``J.T @ r`` -- a scipy sparse matrix (``rosenbrock_problem.jac``) or an ndarray.  Those callables
are user code on NumPy inputs, so ``HostCallableOps`` evaluates them where they live -- once per
trial point (res) and once per accepted iterate (jac), exactly the reference's calls -- and moves
the results to the GPU:

  * the residual vector is uploaded (m doubles), its sum of squares is a device reduction;
  * each Jacobian is uploaded as CSR (32-bit indices) together with the CSR of its transpose;
    J v and J^T w then run in ``gnk_csr_spmv`` with scipy's csr_matvec summation order;
  * the Krylov basis (flat length-n columns), the CGS update, the projected least squares
    (``gnk_flat_gram`` of [J V P^-1 | r] -> lls.CholQR2Solver) and the Armijo trials run in the
    HIP library exactly as for Bratu.

Single GPU (a user callable has no row partition).  The flat Gram runs on MFMA tiles up to 63
basis columns (+ r) and as a transform pass plus a pairwise compensated Gram beyond (up to 1023
columns), so the reference's default -- no restart, the basis growing to max_iter - 1 columns
(ref:gauss_newton_krylow.py:81-82, ref:krylow.py:72-73) -- and dense Jacobians of more than 63
parameters (ref:gauss_newton.py:115-116) run unchanged.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse
import torch

from ._device import make_backend
from .krylow import GeneralizedKrylowSubspaceBreakdown, GeneralizedKrylowSubspaceSpansEntireSpace
from .lls import CholQR2Solver
from .slab import Comm

FLAT_GRAM_KMAX = 1023          # gnk_flat_gram: MFMA tiles up to 63 columns (+ r), a transform + pairwise
                               # Gram pass beyond (KP <= 1024, m x KP doubles in the scratch arena)


class DeviceCSR:
    """A matrix and its transpose as device CSR arrays (int32 indices, fp64 data)."""

    def __init__(self, be, A):
        if scipy.sparse.issparse(A):
            A = A.tocsr()
        else:
            A = scipy.sparse.csr_array(np.asarray(A, dtype=np.float64))
        A = A.astype(np.float64)
        At = A.T.tocsr()
        self.shape = A.shape
        if A.nnz >= 2 ** 31:
            raise ValueError("Jacobian has too many nonzeros for 32-bit CSR indices")
        dev = be.device
        self._arrays = []
        for M in (A, At):
            M.sort_indices()
            self._arrays.append((torch.as_tensor(M.indptr.astype(np.int32), device=dev),
                                 torch.as_tensor(M.indices.astype(np.int32), device=dev),
                                 torch.as_tensor(M.data, device=dev)))
        self._At_data_sq = torch.as_tensor(At.data * At.data, device=dev)   # Jacobi (host squares)
        self.be = be

    def matvec(self, x, y, negate=False):
        ip, ix, d = self._arrays[0]
        self.be.csr_spmv(self.shape[0], ip, ix, d, x, y, negate)

    def rmatvec(self, w, y, negate=False):
        ip, ix, d = self._arrays[1]
        self.be.csr_spmv(self.shape[1], ip, ix, d, w, y, negate)

    def jacobi(self, ones_m, dinv):
        """dinv = 1 / diag(J^T J) (= 1 / diag(A^T A) for A = -J, ref:gauss_newton.py:50-52): the
        squared entries of J^T summed per row in k-ascending order, as scipy's csr_matmat."""
        ip, ix, _ = self._arrays[1]
        self.be.csr_spmv(self.shape[1], ip, ix, self._At_data_sq, ones_m, dinv, reciprocal=True)

    def matmat_rows(self, V, k, W):
        """W[j] = J V[j] for the k basis rows (the reference's ``jac_ev @ krylow.basis``)."""
        for j in range(k):
            self.matvec(V[j], W[j])


PROBE_NMAX = 1 << 16           # operator Jacobians: diag(J^T J) by probing J with unit vectors up to this n


def _host_vec(t):
    return t.detach().cpu().numpy()


class HostOperatorJacobian:
    """``jac(x)`` returned an operator -- a ``scipy.sparse.linalg.LinearOperator`` or any object with
    ``J @ v``, ``J @ V`` and ``J.T @ w`` -- which is all the reference ever does with it
    (ref:gauss_newton_krylow.py:86, ref:krylow.py:62, ref:armijo_goldstein.py:50, ref:gauss_newton.py:36).
    The products run in the user's object on host arrays, with the reference's call shapes (``J @ V`` on
    the (n, k) C-ordered basis, ``J.T @ r``), and their results are uploaded; everything else of the
    loop stays on the device.  Negation is applied on the device (exact, as the reference's ``-J.T @ r``)."""

    def __init__(self, be, J, m, n):
        self.J, self.be = J, be
        shape = getattr(J, "shape", None)
        self.shape = (int(shape[0]), int(shape[1])) if shape is not None else (m, n)

    def _put(self, a, y, negate, what, size):
        a = np.asarray(a, dtype=np.float64).reshape(-1)
        if a.size != size:
            raise ValueError(f"jac(x) {what} returned {a.size} values, expected {size}")
        y.copy_(self.be.to_device(a))
        if negate:
            y.neg_()

    def matvec(self, x, y, negate=False):
        self._put(self.J @ _host_vec(x), y, negate, "@ v", y.numel())

    def rmatvec(self, w, y, negate=False):
        self._put(self.J.T @ _host_vec(w), y, negate, ".T @ w", y.numel())

    def matmat_rows(self, V, k, W):
        Vh = np.ascontiguousarray(_host_vec(V[:k]).T)          # the reference's (n, k) basis layout
        Y = np.asarray(self.J @ Vh, dtype=np.float64)
        if Y.shape != (W.shape[1], k):
            raise ValueError(f"jac(x) @ V returned shape {Y.shape}, expected {(W.shape[1], k)}")
        W[:k].copy_(self.be.to_device(np.ascontiguousarray(Y.T)))

    def jacobi(self, ones_m, dinv):
        """dinv = 1 / diag(J^T J) for ``cg_least_squares``' Jacobi preconditioner (ref:gauss_newton.py:50-54;
        the reference's ``(A.T @ A).diagonal()`` needs a sparse matrix).  The operator is probed with blocks
        of unit vectors (``J @ E``: the columns of J, exactly), and each column's squares are summed in
        ascending row order on the device (gnk_csr_spmv, reciprocal mode) -- the order of the sparse path."""
        n = dinv.numel()
        if n > PROBE_NMAX:
            raise NotImplementedError(f"gauss_newton with an operator Jacobian of {n} columns: diag(J^T J) is "
                                      f"probed column by column up to n = {PROBE_NMAX}; return a sparse matrix, "
                                      "or use generic.Problem with diag_jtj")
        b = max(1, min(256, (1 << 24) // max(1, n)))
        for j0 in range(0, n, b):
            nb = min(b, n - j0)
            E = np.zeros((n, nb))
            E[j0 + np.arange(nb), np.arange(nb)] = 1.0
            Jb = np.asarray(self.J @ E, dtype=np.float64).reshape(-1, nb)
            Bt = scipy.sparse.csr_array(np.ascontiguousarray(Jb.T))          # column j of J as row j
            dev = self.be.device
            ip = torch.as_tensor(Bt.indptr.astype(np.int32), device=dev)
            ix = torch.as_tensor(Bt.indices.astype(np.int32), device=dev)
            dsq = torch.as_tensor(Bt.data * Bt.data, device=dev)
            self.be.csr_spmv(nb, ip, ix, dsq, ones_m, dinv[j0:j0 + nb], reciprocal=True)


def is_operator(J) -> bool:
    """The reference's duck typing of ``jac(x)``: anything with ``@`` and ``.T`` that is not an array."""
    if scipy.sparse.issparse(J) or isinstance(J, np.ndarray) or torch.is_tensor(J):
        return False
    return hasattr(J, "__matmul__") and hasattr(J, "T")


class FlatKrylovBasis:
    """ref:krylow.py:16-73 on flat device vectors (same interface as krylow.DeviceKrylovBasis)."""

    FUSE_KMAX = 0          # no fused first trial for generic problems
    deferred = False       # Gram-Schmidt runs inside update (the breakdown is known there)
    pending = False

    def __init__(self, ops, kmax: int):
        self.ops = ops
        self.be = ops.be
        self.kmax = int(kmax)
        self.V = self.be.zeros(self.kmax, ops.n)
        self.k = 0
        self._c = self.be.zeros(self.kmax)
        self._h = self.be.zeros(self.kmax)
        self._stats = self.be.zeros(2)
        self._g = self.be.zeros(ops.n)

    @property
    def shape(self):
        return (self.ops.n, self.k)

    def gram_k(self):
        return self.k

    def step_scale(self):
        return np.ones(self.k)                     # columns are stored normalised

    def start(self, x):
        """ref:krylow.py:30-39."""
        self.be.flat_stats(x, self._stats)
        sumsq, maxabs = (float(v) for v in self._stats.cpu().numpy())
        if maxabs <= 1e-8:                                    # np.allclose(x0, 0) (:31)
            raise ValueError("x0 is not allowed to be 0 in the gauss_newton_krylow algorithm")
        nrm = math.sqrt(sumsq)                                # :36
        self.be.flat_div(x, nrm, self.V[0])                   # :37
        self.k = 1
        return np.array([nrm])

    def x(self, c: np.ndarray, out):
        k = len(c)
        self._c[:k].copy_(self.be.to_device(c))
        self.be.flat_gemv(self.V, k, self._c, out)
        return out

    def update(self, u_jac, r, it=None, products=None, prod_slot=None, halo=True):
        """ref:krylow.py:55-73 with jac_ev = J(u_jac), res_ev = r (CGS done here, not deferred)."""
        k = self.k
        if k == self.ops.n:                                   # :59-60
            raise GeneralizedKrylowSubspaceSpansEntireSpace
        if k >= self.kmax:
            raise RuntimeError("Krylov basis storage exhausted")
        g = self._g
        self.ops.vjp(u_jac, r, g, negate=True)                # g = -J^T r (:62)
        self.be.flat_gemv_t(self.V, k, g, self._h)            # h = V^T g (:64)
        self.be.flat_cgs_update(self.V, k, self._h, g, self._stats)   # g -= V h (:64)
        sumsq, maxabs = (float(v) for v in self._stats.cpu().numpy())
        if maxabs <= 1e-8 and not math.isnan(sumsq):          # :66
            raise GeneralizedKrylowSubspaceBreakdown(
                "Normal residual is allready inside generalized Krylow Subspcae, there for gauss newton "
                "krylow algorithm has to proceed without enlarging the subspace.")
        nrm = math.sqrt(sumsq)                                # :71
        self.be.flat_div(g, nrm, self.V[k])
        self.k = k + 1


class _IdentityBasis:
    """V = I_n as a basis (the dense least-squares solve: J V = J)."""

    pending = False

    def __init__(self, be, n):
        self.V = be.to_device(np.eye(n))
        self.k = n

    def gram_k(self):
        return self.k

    def gram_left(self):
        return None


class HostCallableOps:
    """Problem side of the GNK loop (gauss_newton_krylow.GNKSolver) for user callables."""

    jacobian_is_free = False       # jac(x) is user code: evaluated exactly where the reference does
    fuse_trial = False

    def __init__(self, res, jac, n: int, args=(), device=None, backend=None, dense_jacobian: bool = True):
        self.be = backend if backend is not None else make_backend(device)
        self.comm = Comm(single=True)
        self.backend = self.be         # the attribute lls.CholQR2Solver reads
        self.dev = None
        self.res, self.jac, self.args = res, jac, tuple(args)
        self.n = self.n_global = int(n)
        self.m = None                  # learnt from the first res / jac evaluation
        self.dense_jacobian = dense_jacobian
        self._J = {}                   # iterate buffer -> DeviceCSR of jac at its value
        self._dense = {}               # iterate buffer -> jac returned a dense ndarray there
        self._lsq = None               # dense least-squares solver of gauss_newton
        self._W = None
        self._st = self.be.zeros(2)

    # -- vectors -------------------------------------------------------------------------
    def load(self, x0):
        x = np.asarray(x0, dtype=np.float64).reshape(-1)
        if x.size != self.n:
            raise ValueError(f"x0 has {x.size} entries, expected {self.n}")
        return self.be.to_device(x)

    def vec(self):
        return self.be.zeros(self.n)

    def rvec(self):
        """A residual buffer; sized by the first res evaluation when m is not known yet."""
        return self.be.zeros(self.m if self.m is not None else 0)

    def to_host(self, x):
        return x.detach().cpu().numpy().copy()

    def own(self, x):
        return x

    # -- problem -------------------------------------------------------------------------
    def residual(self, x, r) -> float:
        """r = res(x, *args) (the user's function); returns sum(r^2) (device reduction)."""
        rh = np.asarray(self.res(self.to_host(x), *self.args), dtype=np.float64).reshape(-1)
        if self.m is None:
            self.m = rh.size
        if r.numel() == 0:
            r.resize_(rh.size)
        if rh.size != r.numel():
            raise ValueError(f"res returned {rh.size} values, expected {r.numel()}")
        r.copy_(self.be.to_device(rh))
        self.be.flat_stats(r, self._st)
        return float(self._st[0].item())

    def on_jacobian(self, u):
        """jac(u, *args) (the user's function) -> device CSR of J and J^T, kept for u's buffer; an
        operator (``is_operator``) is kept as it is and applied through ``@`` / ``.T @``."""
        Jh = self.jac(self.to_host(u), *self.args)
        if is_operator(Jh):
            # the CGLS branch of gauss_newton: the reference's is_sparse test fails for an operator and its
            # lstsq then raises (tests/golden/operator.json); matrix-free J is what CGLS is for
            self._dense[u.data_ptr()] = False
            J = HostOperatorJacobian(self.be, Jh, self.m, self.n)
        else:
            if torch.is_tensor(Jh):
                Jh = Jh.detach().cpu().numpy()
            self._dense[u.data_ptr()] = not scipy.sparse.issparse(Jh)
            J = DeviceCSR(self.be, Jh)
        if J.shape[1] != self.n:
            raise ValueError(f"jac returned shape {J.shape}, expected (m, {self.n})")
        if self.m is None:
            self.m = J.shape[0]
        elif J.shape[0] != self.m:
            raise ValueError(f"jac returned {J.shape[0]} rows, res returned {self.m} values")
        self._J[u.data_ptr()] = J

    def _jac_of(self, u) -> DeviceCSR:
        try:
            return self._J[u.data_ptr()]
        except KeyError:
            raise RuntimeError("no Jacobian evaluated at this iterate") from None

    def jvp(self, u, v, out):
        self._jac_of(u).matvec(v, out)

    def vjp(self, u, w, out, negate=False):
        self._jac_of(u).rmatvec(w, out, negate)

    def max_arena_k(self, with_r=True) -> int:
        """The largest basis size ``gram`` accepts: kp = gram_dim(k, with_r) (k (+ r) rounded up to 16)
        either <= 64 (MFMA tiles, no arena) or with kp * m <= scratch (the wide pass's Y)."""
        kp_max = max(64, (self.be.scratch_doubles() // self.m) // 16 * 16)
        return min(FLAT_GRAM_KMAX, kp_max - (1 if with_r else 0))

    def gram(self, u, V, k, rinv, r, G):
        """Gram of [J(u) V RinvAug | r]: k JVPs into a device W, then gnk_flat_gram."""
        if k > FLAT_GRAM_KMAX:
            raise NotImplementedError(f"generic problems: at most {FLAT_GRAM_KMAX} basis columns per "
                                      "least-squares solve (use krylow_restart)")
        kp = self.be.gram_dim(k, r is not None)
        if kp > 64 and kp * self.m > self.be.scratch_doubles():
            # the wide pass materialises Y = W RinvAug (m x kp) in the library's scratch arena
            raise NotImplementedError(f"generic problems: a {k}-column basis over {self.m} residuals exceeds the "
                                      f"wide Gram's arena ({self.be.scratch_doubles()} doubles; use krylow_restart "
                                      f"<= {self.max_arena_k(r is not None)})")
        if self._W is None or self._W.shape[0] < k:
            self._W = self.be.zeros(max(k, 8), self.m)
        self._jac_of(u).matmat_rows(V, k, self._W)
        self.be.flat_gram(self._W, k, rinv, r, self.m, G)

    # -- Gauss-Newton / CGLS (gauss_newton.GNSolver, DeviceCG) -----------------------------
    def jacobian_is_dense(self, u) -> bool:
        """jac(u) returned an ndarray: gauss_newton takes the lstsq branch (ref:gauss_newton.py:115-116)."""
        return self._dense.get(u.data_ptr(), False)

    def dense_lstsq(self, u, r, d):
        """d = argmin ||-J(u) d - r|| (scipy.linalg.lstsq(-1 * jac_ev, res_ev), ref:gauss_newton.py:116)
        on the device: preconditioned CholeskyQR over the identity basis (the Gram of [J T | r] by
        gnk_flat_gram, T = the previous step's R^-1 when it still conditions J, else CholQR2)."""
        if self.n > FLAT_GRAM_KMAX:
            raise NotImplementedError(f"gauss_newton with a dense Jacobian: at most {FLAT_GRAM_KMAX} parameters "
                                      "(the reference's lstsq branch is for small dense problems, SURVEY §8 f4)")
        if self._lsq is None:
            self._lsq = CholQR2Solver(self, self.n, gram=self.gram, n_global=self.n, device_solve=False)
            self._lsq.quiet = True
            self._lsq.min_norm_if_singular = True
            self._eye = _IdentityBasis(self.be, self.n)
        dh, _, _ = self._lsq.solve(u, self._eye, r)
        d.copy_(self.be.to_device(dh))
        return d
    def jvp_sumsq(self, u, d) -> float:
        """jdd = sum((J(u) d)^2) (ref:armijo_goldstein.py:50)."""
        if getattr(self, "_jd", None) is None:
            self._jd = self.be.zeros(self.m)
        self._jac_of(u).matvec(d, self._jd)
        self.be.flat_stats(self._jd, self._st)
        return float(self._st[0].item())

    def axpy(self, x, t, d, out):
        self.be.flat_axpy(x, t, d, out)

    def sumsq(self, v) -> float:
        self.be.flat_stats(v, self._st)
        return float(self._st[0].item())

    def cg_rhs(self, u, y, b):
        """b = A^T y with A = -J(u): -(J^T y) (ref:gauss_newton.py:46,57)."""
        self._jac_of(u).rmatvec(y, b, negate=True)

    def cg_prepare(self, u):
        self._cgJ = self._jac_of(u)
        if getattr(self, "_tm", None) is None:
            self._tm = self.be.zeros(self.m)
            self._ones = self.be.to_device(np.ones(self.m))
            self._s1 = self.be.zeros(1)
            self._s2 = self.be.zeros(2)

    def cg_jacobi(self, u, dinv):
        self._jac_of(u).jacobi(self._ones, dinv)

    def cg_normal_matvec(self, p, q) -> float:
        """q = A^T (A p) = J^T (J p) (the reference's LinearOperator, ref:gauss_newton.py:36); p . q."""
        self._cgJ.matvec(p, self._tm)
        self._cgJ.rmatvec(self._tm, q)
        self.be.flat_dot(p, q, self._s1)
        return float(self._s1[0].item())

    def cg_update_xr(self, alpha, p, q, x, r, dinv, z):
        self.be.flat_cg_update_xr(alpha, p, q, x, r, dinv, z, self._s2)
        rr, rz = self._s2.cpu().numpy()
        return float(rr), float(rz)

    def cg_update_p(self, beta, first, z, p):
        self.be.flat_cg_update_p(beta, first, z, p)

    def cg_finish(self, x):
        pass

    # -- solver parts --------------------------------------------------------------------
    def make_basis(self, kmax):
        return FlatKrylovBasis(self, kmax)

    def make_lls(self, kmax):
        return CholQR2Solver(self, kmax, gram=self.gram, n_global=self.n, device_solve=False)
