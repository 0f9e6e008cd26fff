"""Row-slab decomposition of the Bratu grid over ranks (one process per GPU).

The reference is single-process; this module is the build's
multi-GPU layer.  Rank p owns global grid rows (the slow x index)
[row0, row0 + nrows); every n-length object -- basis columns, iterates,
residuals, CG vectors -- is split identically and stored as a slab vector with
GHOST rows on each side (include/gnk.h).

Determinism: every cross-rank reduction all-gathers the per-rank partials and
sums them in one fixed pairwise order (``tree_sum``) on every rank, so the control
decisions (Armijo, breakdown, convergence, restart) are bit-identical on all ranks.
With reduction segments (``Comm(segments=...)``, gnk_set_segments) the library reduces
fixed global row segments of N / 8 rows with a decomposition of their own and folds a
rank's segments in the same pairwise order, so a run on 1, 2, 4 or 8 ranks gives the
same bits: the rank values are exactly the subtrees of the one-rank fold.

Collectives: only two kinds exist on the data path --
  * halo: P2P send/recv of GHOST boundary rows to the two neighbours, once per
    appended basis column (and per CG iteration for the search direction);
  * small all-gathers (Gram matrices, V^T g, norms), <= (k+1)^2 doubles.
With world_size == 1 both are no-ops.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

from ._native import GHOST


SEGMENTS_PER_GRID = 8      # reduction segments of N / 8 rows: rank-count invariance for world | 8


def tree_sum(parts):
    """Sum of the rows of ``parts`` (P x n) in the fixed pairwise order v[i] += v[i + w] for
    w = 1, 2, 4, .. (i a multiple of 2w, i + w < P): the balanced binary tree for a power-of-two P,
    and the order of gnk_rank_sum and of gnk_set_segments' segment fold."""
    v = [np.array(parts[p], dtype=np.float64, copy=True) for p in range(parts.shape[0])]
    w = 1
    while w < len(v):
        for i in range(0, len(v) - w, 2 * w):
            v[i] = v[i] + v[i + w]
        w *= 2
    return v[0]


def reduction_segments(N: int, world: int, want) -> int:
    """Rows per reduction segment for a grid of N rows on ``world`` ranks (0 = none): N / 8 when
    segments are wanted (``want`` True, or None and world > 1) and every rank holds whole segments
    (N % 8 == 0 and world divides 8)."""
    on = (world > 1) if want is None else bool(want)
    if not on or N % SEGMENTS_PER_GRID != 0 or SEGMENTS_PER_GRID % world != 0:
        return 0
    return N // SEGMENTS_PER_GRID


def row_partition(N: int, world: int, rank: int):
    """Contiguous, balanced split of N rows over `world` ranks -> (row0, nrows)."""
    base, rem = divmod(N, world)
    nrows = base + (1 if rank < rem else 0)
    row0 = rank * base + min(rank, rem)
    return row0, nrows


class Comm:
    """Rank-ordered reductions and halo exchange over torch.distributed (RCCL on
    GPUs, gloo on CPU).  ``group=None`` with no initialised process group means a
    single rank."""

    def __init__(self, group=None, single: bool = False, segments=None):
        # reduction segments (rank-count-independent reductions, gnk_set_segments): None = on when
        # there is more than one rank, True / False = always / never
        self.segments = segments
        if not single and dist.is_available() and dist.is_initialized():
            self.group = group
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
            # gloo moves device tensors only through host copies (no P2P on GPU memory):
            # stage through the host then (used to rehearse several ranks on one GPU)
            self.stage = dist.get_backend(group) == "gloo"
        else:
            self.group = None
            self.rank, self.world = 0, 1
            self.stage = False
        # device-side sum (tree_sum's order) of all-gathered partials (one kernel, set by the device
        # backend: HipBackend.rank_sum); None: elementwise torch adds in the same order
        self.device_rank_sum = None
        # traffic counters (what one outer step costs in collectives and host waits):
        # all-gathers and their per-rank payload, P2P exchanges and their bytes sent, host waits on
        # device results (a blocking read: the host cannot run ahead of the GPU there)
        self.counters = {"all_gather": 0, "all_gather_bytes": 0, "p2p": 0, "p2p_bytes": 0, "host_wait": 0}

    def _sum_parts_device(self, gath: torch.Tensor, n: int) -> torch.Tensor:
        if self.device_rank_sum is not None:
            out = torch.empty(n, dtype=gath.dtype, device=gath.device)
            return self.device_rank_sum(gath, self.world, out)
        parts = gath.view(self.world, -1)
        v = [parts[p].clone() for p in range(self.world)]
        w = 1
        while w < len(v):                                   # tree_sum's order
            for i in range(0, len(v) - w, 2 * w):
                v[i].add_(v[i + w])
            w *= 2
        return v[0]

    # -- transport: the two collectives of the data path (RCCL on GPUs, gloo on CPU) ---------
    def _count_gather(self, t: torch.Tensor):
        self.counters["all_gather"] += 1
        self.counters["all_gather_bytes"] += t.numel() * t.element_size()

    def _all_gather_into(self, buf: torch.Tensor, t: torch.Tensor):
        dist.all_gather_into_tensor(buf, t, group=self.group)

    def _p2p(self, ops):
        """ops: (dist.isend | dist.irecv, tensor, peer) -> one batched P2P exchange, waited for."""
        reqs = dist.batch_isend_irecv([dist.P2POp(op, t, peer, self.group) for op, t, peer in ops])
        for req in reqs:
            req.wait()

    # -- reductions -------------------------------------------------------------
    def _gather(self, t: torch.Tensor) -> np.ndarray:
        if t.device.type != "cpu":
            self.counters["host_wait"] += 1
        if self.world == 1:
            return t.detach().to("cpu", torch.float64).numpy()[None]
        t = t.contiguous().reshape(-1)
        if self.stage:
            t = t.to("cpu")
        buf = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
        self._count_gather(t)
        self._all_gather_into(buf, t)
        return buf.to("cpu").numpy().reshape(self.world, -1)

    @staticmethod
    def merge_pairs(parts: np.ndarray) -> np.ndarray:
        """Rank-ordered compensated sum of per-rank unevaluated pairs: parts[p] = [s_0, c_0, s_1, c_1,
        ...] (gnk_set_reduce_pairs).  The s are added with TwoSum in rank order, their rounding errors
        and the c are accumulated beside them, and the result is rounded once at the end
        (Ogita-Rump-Oishi Sum2): the device's Dot2 accuracy carried across ranks.  One rank: s + c,
        the value the device itself returns without pairs."""
        S = parts[0, 0::2].copy()
        C = parts[0, 1::2].copy()
        for p in range(1, parts.shape[0]):
            sp, cp = parts[p, 0::2], parts[p, 1::2]
            x = S + sp
            z = x - S
            err = (S - (x - z)) + (sp - z)
            S = x
            C = C + (err + cp)
        return S + C

    def sum_pairs(self, t: torch.Tensor, nq: int) -> np.ndarray:
        """nq compensated per-rank sums given as (s, c) pairs in t[:2 nq] -> their sums over ranks."""
        return self.merge_pairs(self._gather(t[:2 * nq]))

    def sum(self, t: torch.Tensor) -> np.ndarray:
        """Sum of a small per-rank tensor over ranks, in tree_sum's order (host result)."""
        return tree_sum(self._gather(t))

    def sum_max(self, t: torch.Tensor) -> tuple[float, float]:
        """t = [sum, max] per rank -> (sum over ranks, NaN-propagating max over ranks)."""
        sums, m = self.sum_and_max(t, 1)
        return float(sums[0]), m

    def sum_max_pairs(self, t: torch.Tensor, n: int) -> list:
        """t = [s_0, m_0, s_1, m_1, ..] (n [sum, max] pairs) per rank -> [(sum over ranks, NaN-propagating
        max over ranks)] * n: ``sum_max``'s arithmetic for each pair, several of them in one collective and
        one host read."""
        parts = self._gather(t[:2 * n])
        sums = tree_sum(parts[:, 0::2])
        out = []
        for i in range(n):
            m = float(parts[0][2 * i + 1])
            for p in range(1, parts.shape[0]):
                v = float(parts[p][2 * i + 1])
                if v > m or math.isnan(v):
                    m = v
            out.append((float(sums[i]), m))
        return out

    def sum_and_max(self, t: torch.Tensor, nsum: int) -> tuple[np.ndarray, float]:
        """t = [s_0 .. s_{nsum-1}, m] per rank -> (sums over ranks, NaN-propagating max): several
        control scalars of one step in one collective and one host read."""
        parts = self._gather(t)
        s = tree_sum(parts[:, :nsum])
        m = float(parts[0][nsum])
        for p in range(1, parts.shape[0]):
            v = float(parts[p][nsum])
            if v > m or math.isnan(v):
                m = v
        return s, m

    def sum_except_max(self, t: torch.Tensor, imax: int, shared: torch.Tensor = None):
        """Rank-ordered sums of every entry of a small per-rank tensor except entry ``imax``, which
        is the NaN-propagating max over ranks: a step's control scalars in one collective.  With
        ``shared`` (a device buffer identical on every rank) -> (sums, host copy of shared), read in
        the same device-to-host copy on one rank."""
        if shared is not None:
            n = t.numel()
            if self.world == 1:
                both = torch.cat([t.reshape(-1), shared.reshape(-1)]).to("cpu", torch.float64).numpy()
                return both[:n].copy(), both[n:].copy()
            return self.sum_except_max(t, imax), shared.to("cpu", torch.float64).numpy().copy()
        parts = self._gather(t)
        s = tree_sum(parts)
        m = float(parts[0][imax])
        for p in range(1, parts.shape[0]):
            v = float(parts[p][imax])
            if v > m or math.isnan(v):
                m = v
        s[imax] = m
        return s

    # -- asynchronous read of a step's control scalars ------------------
    def read_async(self, t: torch.Tensor, shared: torch.Tensor = None, pinned: torch.Tensor = None):
        """Enqueue the cross-rank gather of a small per-rank device tensor ``t`` (and a copy of
        ``shared``, identical on every rank) into host memory; returns a handle for ``complete``
        (the host does not wait here).  ``device_sum(handle)``: the sum over ranks on the device,
        for device-side consumers that must not wait for the host."""
        n = t.numel()
        m = shared.numel() if shared is not None else 0
        on_gpu = t.device.type != "cpu" and pinned is not None
        if not on_gpu or (self.world > 1 and self.stage):
            parts = self._gather(t)
            sh = shared.detach().to("cpu", torch.float64).numpy().copy() if shared is not None else None
            return _ReadHandle(None, None, n, parts, sh, t)
        if self.world == 1:
            gath = t.reshape(-1)
            if (shared is not None and shared.untyped_storage().data_ptr() == gath.untyped_storage().data_ptr()
                    and shared.storage_offset() >= gath.storage_offset() + n and shared.is_contiguous()):
                # the pack and the solve's output share one device buffer (lls._LSBuffers.comb): one copy of
                # the span from the pack's start to the output's end instead of two
                base = gath.storage_offset()
                span = shared.storage_offset() + m - base
                src = torch.as_strided(gath, (span,), (1,), base)
                host = pinned[:span]
                host.copy_(src, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(t.device))
                return _ReadHandle(host, ev, n, None, None, gath, shared.storage_offset() - base)
        else:
            gath = torch.empty(self.world * n, dtype=t.dtype, device=t.device)
            self._count_gather(t)
            self._all_gather_into(gath, t.contiguous().reshape(-1))
        wn = self.world * n
        host = pinned[:wn + m]
        host[:wn].copy_(gath, non_blocking=True)
        if shared is not None:
            host[wn:].copy_(shared.reshape(-1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(t.device))
        return _ReadHandle(host, ev, n, None, None, gath, wn if shared is not None else None)

    def device_sum(self, h) -> torch.Tensor:
        """Sum over ranks (on the device) of the tensor behind a read handle."""
        if self.world == 1:
            return h.gath
        if h.gath.numel() == h.n:                 # staged / CPU path: sum on the host, copy back
            return torch.from_numpy(self._rank_sum(h.parts)).to(h.gath.device)
        return self._sum_parts_device(h.gath, h.n)

    @staticmethod
    def _rank_sum(parts):
        return tree_sum(parts)

    def complete(self, h, imax: int):
        """Wait for a read handle -> (sums over ranks except entry ``imax``: NaN-propagating max
        over ranks, shared host copy or None)."""
        if h.ev is not None:
            self.counters["host_wait"] += 1
            h.ev.synchronize()
            wn = self.world * h.n
            a = h.host.numpy()
            h.parts = a[:wn].reshape(self.world, h.n).copy()
            h.shared = a[h.soff:].copy() if h.soff is not None else None
        parts = h.parts
        s = self._rank_sum(parts)
        m = float(parts[0][imax])
        for p in range(1, parts.shape[0]):
            v = float(parts[p][imax])
            if v > m or math.isnan(v):
                m = v
        s[imax] = m
        return s, h.shared

    def sum_device(self, t: torch.Tensor) -> torch.Tensor:
        """Sum over ranks of a small per-rank device tensor, left on the device (no host round
        trip on RCCL): the same IEEE additions in the same order as ``sum``."""
        if self.world == 1:
            return t
        if self.stage:
            return torch.from_numpy(self.sum(t)).to(t.device)
        t = t.contiguous().reshape(-1)
        buf = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
        self._count_gather(t)
        self._all_gather_into(buf, t)
        return self._sum_parts_device(buf, t.numel())

    def gather_device(self, t: torch.Tensor) -> torch.Tensor:
        """The ranks' copies of a small per-rank tensor, rank-major in one tensor on ``t``'s device
        ([world * n]): a device all-gather on RCCL (no host wait); staged through the host on gloo."""
        t = t.contiguous().reshape(-1)
        if self.world == 1:
            return t
        if self.stage:
            return torch.from_numpy(self._gather(t).reshape(-1).copy()).to(t.device)
        buf = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
        self._count_gather(t)
        self._all_gather_into(buf, t)
        return buf

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    # -- halo -------------------------------------------------------------------
    def halo(self, vec: torch.Tensor, N: int, nrows: int):
        """Fill the GHOST ghost rows of a slab vector from the neighbouring ranks."""
        if self.world == 1:
            return
        g = GHOST * N
        own_end = (GHOST + nrows) * N
        staged = self.stage and vec.device.type != "cpu"
        host = vec.to("cpu") if staged else vec
        ops = []
        if self.rank > 0:
            ops.append((dist.isend, host[g:2 * g], self.rank - 1))
            ops.append((dist.irecv, host[0:g], self.rank - 1))
        if self.rank < self.world - 1:
            ops.append((dist.isend, host[own_end - g:own_end], self.rank + 1))
            ops.append((dist.irecv, host[own_end:own_end + g], self.rank + 1))
        self.counters["p2p"] += 1
        self.counters["p2p_bytes"] += sum(t.numel() * t.element_size() for op, t, _ in ops if op is dist.isend)
        self._p2p(ops)
        if staged:
            if self.rank > 0:
                vec[0:g].copy_(host[0:g])
            if self.rank < self.world - 1:
                vec[own_end:own_end + g].copy_(host[own_end:own_end + g])

    def gather_rows(self, owned: torch.Tensor, N: int) -> np.ndarray:
        """All ranks' owned rows -> the full host vector (variable slab sizes): one tensor
        all-gather of the owned rows, each rank's part padded to the largest slab."""
        if self.world == 1:
            return owned.detach().to("cpu").numpy().copy()
        sizes = [row_partition(N, self.world, p)[1] * N for p in range(self.world)]
        big = max(sizes)
        dev = torch.device("cpu") if self.stage else owned.device
        pad = torch.zeros(big, dtype=torch.float64, device=dev)
        pad[:owned.numel()] = owned.detach().reshape(-1)
        buf = torch.empty(self.world * big, dtype=torch.float64, device=dev)
        self._all_gather_into(buf, pad)
        del pad
        parts = buf.view(self.world, big)
        return torch.cat([parts[p, :sizes[p]] for p in range(self.world)]).to("cpu").numpy()


class SlabVector:
    """A vector already distributed as this rank's slab (owned rows + GHOST rows each side, ghost
    rows valid): accepted wherever a full-grid host vector is, without any whole-grid copy
    (``inputs.slab_inputs`` builds the bench workload this way)."""

    __slots__ = ("data",)

    def __init__(self, data: torch.Tensor):
        self.data = data


class _ReadHandle:
    __slots__ = ("host", "ev", "n", "parts", "shared", "gath", "soff")

    def __init__(self, host, ev, n, parts, shared, gath, soff=None):
        self.host, self.ev, self.n, self.parts, self.shared, self.gath = host, ev, n, parts, shared, gath
        self.soff = soff                      # where the shared buffer's copy starts in ``host``


class Slab:
    """Geometry of this rank's slab + helpers to move whole-grid host arrays in and out."""

    def __init__(self, N: int, comm: Comm):
        self.N = int(N)
        self.comm = comm
        if comm.world > N // GHOST:
            raise ValueError(f"grid of {N} rows cannot be split over {comm.world} ranks "
                             f"(each rank needs >= {GHOST} rows)")
        self.row0, self.nrows = row_partition(self.N, comm.world, comm.rank)
        self.length = (self.nrows + 2 * GHOST) * self.N
        self.own = slice(GHOST * self.N, (GHOST + self.nrows) * self.N)
        self.n_global = self.N * self.N

    def from_host(self, full, backend) -> torch.Tensor:
        """Slab vector (owned + up to GHOST rows each side) from a full-grid vector (or a copy of a
        SlabVector of this geometry)."""
        if isinstance(full, SlabVector):
            if full.data.numel() != self.length:
                raise ValueError(f"SlabVector of length {full.data.numel()}, this rank's slab has {self.length}")
            out = backend.zeros(self.length)
            out.copy_(full.data.reshape(-1))
            return out
        full = torch.as_tensor(np.asarray(full, dtype=np.float64) if not torch.is_tensor(full) else full)
        out = backend.zeros(self.length)
        lo = max(self.row0 - GHOST, 0)
        hi = min(self.row0 + self.nrows + GHOST, self.N)
        dst0 = (lo - (self.row0 - GHOST)) * self.N
        out[dst0:dst0 + (hi - lo) * self.N] = full.reshape(-1)[lo * self.N:hi * self.N].to(out.device, torch.float64)
        return out

    def to_host(self, slab_vec: torch.Tensor) -> np.ndarray:
        """Full-grid host vector gathered from every rank's owned rows."""
        return self.comm.gather_rows(slab_vec[self.own], self.N)
