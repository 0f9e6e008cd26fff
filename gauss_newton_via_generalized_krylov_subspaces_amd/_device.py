"""Device state shared by the solvers: backend + slab geometry + problem setup."""
from __future__ import annotations

import torch

from ._native import HipBackend
from .slab import Comm, Slab, reduction_segments


def default_device():
    if not torch.cuda.is_available():
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def make_backend(device=None):
    """The product backend: HIP only (raises when libgnk.so or the GPU is missing)."""
    return HipBackend(device if device is not None else default_device())


class BratuDevice:
    """One rank's view of a Bratu problem: backend configured for its slab."""

    def __init__(self, problem, comm: Comm | None = None, device=None, backend=None):
        self.problem = problem
        self.comm = comm or Comm()
        self.backend = backend if backend is not None else make_backend(device)
        self.slab = Slab(problem.N, self.comm)
        self.backend.set_bratu(problem.N, self.slab.row0, self.slab.nrows, problem.grid_resolution,
                               problem.ALPHA, problem.LAMBDA)
        if self.backend.slab_len() != self.slab.length:
            raise RuntimeError("slab length mismatch between host and libgnk")
        # rank-count-independent reductions (slab.reduction_segments; on by default for several ranks)
        self.seg_rows = reduction_segments(problem.N, self.comm.world, getattr(self.comm, "segments", None))
        if hasattr(self.backend, "set_segments"):
            self.backend.set_segments(self.seg_rows)
        if self.comm.world > 1 and not self.comm.stage and hasattr(self.backend, "rank_sum"):
            self.comm.device_rank_sum = self.backend.rank_sum

    def vec(self):
        return self.backend.zeros(self.slab.length)

    def load(self, full):
        return self.slab.from_host(full, self.backend)

    def scalar(self, n=1):
        return self.backend.zeros(n)


class DeviceIterate:
    """What a solver callback receives with ``callback_format="device"``: this rank's slab vector
    of the iterate (valid on owned +-GHOST rows) and the solver's sum of squares of the residual
    at it (over all ranks), so per-iteration diagnostics need no host copy of x."""

    __slots__ = ("x", "sumsq", "ops")

    def __init__(self, x, sumsq, ops):
        self.x, self.sumsq, self.ops = x, sumsq, ops


class SingleRankOperator:
    """Evaluate F, J v, J^T w, diag(J^T J) on whole-grid host arrays (one rank) --
    the drop-in behaviour of the reference closures."""

    def __init__(self, problem, device=None):
        self.dev = BratuDevice(problem, Comm(single=True), device)

    def _in(self, a):
        return self.dev.load(a if not torch.is_tensor(a) else a.detach().cpu().numpy())

    def _out(self, t):
        return t[self.dev.slab.own].cpu().numpy()

    def forward(self, u):
        F = self.dev.vec()
        self.dev.backend.forward(self._in(u), F)
        return self._out(F)

    def jvp(self, u, v):
        out = self.dev.vec()
        self.dev.backend.jvp(self._in(u), self._in(v), out)
        return self._out(out)

    def vjp(self, u, w):
        out = self.dev.vec()
        self.dev.backend.vjp(self._in(u), self._in(w), out)
        return self._out(out)

    def diag_jtj(self, u):
        out = self.dev.vec()
        self.dev.backend.diag_jtj(self._in(u), out)
        return self._out(out)
