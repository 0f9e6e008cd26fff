"""Per-rank staging of the synthetic Bratu workload (ref:bratu_pde_test.py:22-36) for large grids.

The reference builds the whole grid on one host: u_true (ref:bratu_pde_problem.py:69-74),
y = pde_operator(u_true), u0 = u_true + 0.1 N(0, 1) with ``np.random.seed(42)``.  At 32768^2 one
such vector is 8.6 GB, so building all of them on every rank (and evaluating F over the whole
grid on every GPU) does not scale to the 8-GPU C4 configuration.  Here each rank only ever holds
its own slab (owned rows + GHOST rows each side):

  * u_true rows are evaluated directly (the same elementwise exp(-10 (x^2 + y^2)) on the same
    linspace nodes, so bit-identical to the full-grid array);
  * u0's normal draws are streamed through the legacy MT19937 generator in bounded chunks and only
    this slab's rows are kept (chunked draws continue the same sequence, so the values are those of
    the reference's single ``np.random.normal(size=n)`` call);
  * y = F(u_true) runs the forward stencil kernel on the slab; its ghost rows come from the
    neighbours by the halo exchange every basis column uses.

The results are ``SlabVector`` objects, which the solvers take wherever the reference takes a
full-grid vector (``GNKSolver(problem, y)``, ``setup(x0)``, ``GNSolver``).
"""
from __future__ import annotations

import numpy as np
import torch

from ._native import GHOST
from .bratu_pde_problem import default_u
from .slab import SlabVector

CHUNK = 1 << 24             # normal draws per chunk (128 MiB of float64)


def u_true_rows(problem, lo: int, hi: int) -> np.ndarray:
    """Rows [lo, hi) (slow x index) of ``problem.u_true`` (flat index jx * N + iy)."""
    if problem.u is not default_u:                    # a user u(x1, x2): the full-grid property
        return problem.u_true[lo * problem.N:hi * problem.N]
    lin = np.linspace(problem.lower_bound, problem.upper_bound, problem.grid_nodes + 1)[1:-1]
    xx = lin[lo:hi, None]
    yy = lin[None, :]
    return np.exp(-10 * (xx ** 2 + yy ** 2)).reshape(-1)


def normal_rows(seed: int, N: int, lo: int, hi: int) -> np.ndarray:
    """Entries [lo N, hi N) of ``np.random.seed(seed); np.random.normal(0, 1, N * N)``, drawing the
    sequence in chunks of at most CHUNK values and keeping only this range."""
    rs = np.random.RandomState(seed)
    a, b = lo * N, hi * N
    pos = 0
    while pos + CHUNK <= a:                            # skip whole chunks before the range
        rs.normal(loc=0, scale=1, size=CHUNK)
        pos += CHUNK
    if a > pos:
        rs.normal(loc=0, scale=1, size=a - pos)
    return rs.normal(loc=0, scale=1, size=b - a)


def _slab_rows(slab):
    lo = max(slab.row0 - GHOST, 0)
    hi = min(slab.row0 + slab.nrows + GHOST, slab.N)
    return lo, hi, (lo - (slab.row0 - GHOST)) * slab.N


def slab_inputs(dev, seed: int = 42, noise: float = 0.1):
    """(u0, y, u_true) of the bench workload as this rank's slab vectors (``dev``: a BratuDevice)."""
    problem, slab, be = dev.problem, dev.slab, dev.backend
    lo, hi, off = _slab_rows(slab)
    ut_host = u_true_rows(problem, lo, hi)
    u_true = be.zeros(slab.length)
    u_true[off:off + ut_host.size] = torch.from_numpy(ut_host).to(u_true.device)
    u0 = be.zeros(slab.length)
    u0_host = ut_host + noise * normal_rows(seed, slab.N, lo, hi)   # u_true + 0.1 * N(0, 1)
    u0[off:off + u0_host.size] = torch.from_numpy(u0_host).to(u0.device)
    del ut_host, u0_host
    y = be.zeros(slab.length)
    be.forward(u_true, y)                                 # owned rows
    dev.comm.halo(y, slab.N, slab.nrows)                   # ghost rows from the neighbours
    return SlabVector(u0), SlabVector(y), SlabVector(u_true)
