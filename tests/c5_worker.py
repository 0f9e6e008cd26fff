"""C5's basis growth to k = 200 on 8 ranks, rehearsed on ONE GPU ("run k = 200 on 8 GPUs as the
MFMA stress"; BASELINE configs[4]).

C5 itself is Bratu 16384^2 with no restart (ref:gauss_newton_krylow.py:81-82: krylow_restart = max_iter,
ref:krylow.py:72-73 appends a column per iteration) to k = 200: its basis is 201 x 2.15 GB = 429 GB, which
needs the 8 GPUs' HBM.  Eight ranks sharing cuda:0 hold the same total, so the rehearsal runs the same
algorithm at 8192^2 (V = 201 x 537 MB = 108 GB): every Gram kernel of the wide path in turn -- staged MFMA
(k <= 31, the 4x4x4-block k_gram_q from k = 8), the marching wide pass (32..111) and the pair-split k_gram
(112..200) -- with the (k+1)^2 Grams all-gathered and rank-summed, the host least-squares solve past the
device solve's 32 columns, and the unfused trial / update kernels past the fused trial's 24 columns.
Collectives go through slab.Comm's RCCL branches on the host-staged transport (tests/transport_shim.py);
every rank stages only its slab of the inputs.  Then rank 0 runs the same solve on one rank over the whole
grid.  Reported (rank 0 writes --out):
  * identical decisions and per-iteration scalars on every rank;
  * 8 ranks vs 1 rank, both with reduction segments (gnk_set_segments): nit / nrev / njev, per-iteration
    nfev and basis size, stdout; per-iteration ||x_k|| and ||r_k|| relative differences -- bit for bit while
    the basis is on the segmented kernels (k <= 31), then differing by rounding: the wide Gram kernels
    (k > 31) reduce over their own slab decomposition (the numbers are recorded, not asserted);
  * the one-rank run's reference basis (sc_j V_j) orthonormal: max |V^T V - I| (gnk_flat_gemv_t);
  * seconds per run and the Gram pass per k (the one-rank run's HIP-event timer).

  python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node 8 tests/c5_worker.py \
      --out c5.json
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402
from tests.transport_shim import StagedTransportComm  # noqa: E402


def log(msg):
    r = dist.get_rank() if dist.is_initialized() else 0
    print(f"[rank {r} {time.strftime('%X')}] {msg}", file=sys.stderr, flush=True)


def solve(N, comm, iters, orth=False):
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    dev = BratuDevice(prob, comm)
    u0, y, ut = slab_inputs(dev)
    del ut
    rec = {"xnorm2": [], "rsumsq": [], "nfev": []}
    st = dev.backend.zeros(4)

    def cb(x, nfev, cg_iter):
        dev.backend.vec_stats(x.x, st)
        rec["xnorm2"].append(float(comm.sum(st[:1])[0]))
        rec["rsumsq"].append(float(x.sumsq))
        rec["nfev"].append(int(nfev))
        if len(rec["nfev"]) % 20 == 0:
            log(f"it {len(rec['nfev'])}: k {s.basis.k} nfev {nfev} ||x||^2 {rec['xnorm2'][-1]!r}")

    # no restart: krylow_restart = max_iter (ref:gauss_newton_krylow.py:81-82)
    s = gnk.GNKSolver(prob, y, krylow_restart=None, max_iter=iters + 1, comm=comm, backend=dev.backend,
                      callback=cb, callback_format="device")
    buf = io.StringIO()
    t0 = time.time()
    with contextlib.redirect_stdout(buf):
        s.setup(u0)
        del u0
        while not s.step():
            pass
        r = s.finish(result_format="torch")
    torch.cuda.synchronize()
    secs = time.time() - t0
    out = {"nit": r.nit, "nrev": r.nrev, "njev": r.njev, "success": bool(r.success), **rec,
           "k": [t["k"] for t in s.trace], "trials": [t["trials"] for t in s.trace], "stdout": buf.getvalue(),
           "max_cond": max((h[2][-1] for h in s.lls.history if h[2]), default=None),
           "multi_pass_solves": sum(1 for h in s.lls.history if h[1] > 1), "seconds": secs,
           "segment_fallbacks": dev.backend.segment_fallbacks()}
    if orth:
        b, be = s.basis, dev.backend
        k = b.k
        h = be.zeros(k)
        G = np.zeros((k, k))
        for j in range(k):
            be.flat_gemv_t(b.V, k, b.V[j], h)
            G[:, j] = h.cpu().numpy()
        sc = b.sc[:k]
        G = sc[:, None] * G * sc[None, :]
        out["basis_k"] = k
        out["max_abs_VtV_minus_I"] = float(np.max(np.abs(G - np.eye(k))))
    del s, r, y, dev, st
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    log(f"multi-rank solve, grid {a.grid}, world {world}, {a.iters} iterations without restart")
    comm = StagedTransportComm()
    mine = solve(a.grid, comm, a.iters)
    log(f"multi-rank done in {mine['seconds']:.1f} s: nit {mine['nit']} nrev {mine['nrev']} max k {max(mine['k'])}")
    every = [None] * world
    dist.all_gather_object(every, mine)
    dist.barrier()
    if rank != 0:
        dist.barrier()
        dist.destroy_process_group()
        return 0
    log("single-rank solve over the whole grid")
    try:
        one = solve(a.grid, Comm(single=True, segments=True), a.iters, orth=True)
        log(f"single-rank done in {one['seconds']:.1f} s")
    except Exception as e:
        log(f"single-rank solve raised {type(e).__name__}: {e}")
        one = {"error": f"{type(e).__name__}: {e}", "xnorm2": [], "rsumsq": []}
    dist.barrier()
    ranks_identical = all({k: v for k, v in e.items() if k != "seconds"} ==
                          {k: v for k, v in mine.items() if k != "seconds"} for e in every)
    keys = ("nit", "nrev", "njev", "success", "nfev", "k", "trials", "stdout")
    same = all(mine[k] == one.get(k) for k in keys)

    def rel(a_, b_):
        a_, b_ = np.sqrt(np.array(a_)), np.sqrt(np.array(b_))
        return (np.abs(a_ - b_) / np.abs(b_)).tolist() if len(a_) == len(b_) and len(b_) else [float("inf")]

    ex, er = rel(mine["xnorm2"], one["xnorm2"]), rel(mine["rsumsq"], one["rsumsq"])
    rep = {"grid": a.grid, "world": world, "iters": a.iters, "max_k": max(mine["k"]),
           "ranks_identical": ranks_identical, "bookkeeping_equal": same,
           "max_rel_xnorm_diff": max(ex), "max_rel_rnorm_diff": max(er), "rel_xnorm_diff": ex,
           "rel_rnorm_diff": er, "single_max_abs_VtV_minus_I": one.get("max_abs_VtV_minus_I"),
           "single_basis_k": one.get("basis_k"), "max_cond_multi": mine["max_cond"],
           "max_cond_single": one.get("max_cond"), "seconds_multi": mine["seconds"],
           "seconds_single": one.get("seconds"), "shim_calls": dict(comm.staged_calls),
           "multi": {k: v for k, v in mine.items() if k != "stdout"},
           "single": {k: v for k, v in one.items() if k != "stdout"}}
    with open(a.out, "w") as f:
        json.dump(rep, f, indent=1)
    log(json.dumps({k: rep[k] for k in ("ranks_identical", "bookkeeping_equal", "max_rel_xnorm_diff",
                                        "max_rel_rnorm_diff", "single_max_abs_VtV_minus_I", "max_k")}))
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
