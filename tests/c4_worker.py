"""C4 at its size on ONE GPU: Bratu 32768^2 row-partitioned over 8 ranks (BASELINE configs[3]).

All ranks share cuda:0 (RCCL refuses several ranks on one device), so the collectives go through
the host-staged transport of tests/transport_shim.py -- slab.Comm's RCCL branches with gloo moving
the bytes.  Every rank stages only its own slab of the inputs (inputs.slab_inputs: u0's normal draws
streamed, y = F(u_true) by the forward kernel + halo), runs GNKSolver at krylow_restart = 20 (C4's
restart) for ITERS outer iterations (ref:gauss_newton_krylow.py:84-136) and keeps only scalars; then every rank
frees its state and rank 0 runs the same solve on one rank over the whole grid.  Checked
(rank 0 writes --out):
  * every rank took identical decisions and holds identical per-iteration scalars;
  * 8 ranks vs 1 rank, both with reduction segments of N / 8 rows (slab.reduction_segments: on by
    default for several ranks, asked for on the one rank): nit / nrev / njev / success, per-iteration
    nfev, basis sizes, stdout AND the per-iteration ||x_k||^2 (gnk_vec_stats, segment-reduced) and
    ||r_k||^2 (the solver's own) bit for bit -- every reduction of the GNK path is rank-count
    independent (gnk_set_segments).  Without segments (round 3) ||x_k|| differed by up to 6.8e-8 at
    iteration 1, where the step cancels ||x_0|| ~ 3e3 to ||x_1|| ~ 5e-6 (ref:gauss_newton_krylow.py:98):
    the relative differences and the bound that covered them (max(1e-10, CANCEL u ||x_0|| / ||x_k||,
    cycle_spread_k)) are still reported.
Then GN + CGLS at the same size and partition ("C3 at 32768^2"; ref:gauss_newton.py:11-60,
63-138): GN_ITERS outer iterations, Jacobi CGLS at rtol 1e-8 capped at CG_MAXITER iterations per solve,
8 ranks vs 1 rank.  The CG scalars and ||.||^2 are compensated pairs merged across ranks before one
rounding (slab.Comm.sum_pairs), so cg_iter, nfev and the per-iteration ||x_k||^2 (the solver's own
compensated sum) must agree bit for bit; ||r_k||^2 is a plain rank-ordered sum, within 1e-10.
Memory: ITERS = 6 iterations hold at most 7 basis columns (+ ~9 vectors) x 8.6 GB ~ 140 GB, on 8
ranks or on one.  (A restart inside the window would make the next step a k = 1 step whose Armijo
test compares two sums of 1e9 squares differing by less than their rounding: the reference's own
arithmetic decides it by noise at this size, so the window stays inside the first restart cycle.)

  python -m torch.distributed.run --standalone --nproc-per-node 8 tests/c4_worker.py --out c4.json
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
from gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton import GNSolver  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402
from tests.transport_shim import StagedTransportComm  # noqa: E402

TOL = 1e-10
CANCEL = 16          # roundings of size u ||x_0|| allowed in x_k
U = np.finfo(np.float64).eps / 2


def cycle_spread(n):
    """2 |exact_k1_i - base_i| / |base_i| of the pinned 8192^2 restart-cycle fixture (tests/golden/
    make_cycle8192.py, the same workload family and restart): how far the reference's own trajectory
    moves when only its cancellation-limited k = 1 dot products are rounded differently.  At 32768^2 that
    cancellation is ~19x deeper (||x_1|| / ||x_0|| = 1.7e-9 vs 3.2e-8), so as a bound here it is conservative."""
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "large_cycle8192.json")) as f:
        v = json.load(f)["variants"]
    b, e = np.array(v["base"]["xnorm"][:n]), np.array(v["exact_k1"]["xnorm"][:n])
    return 2 * np.abs(e - b) / np.abs(b)


def log(msg):
    print(f"[rank {dist.get_rank()} {time.strftime('%X')}] {msg}", file=sys.stderr, flush=True)


def solve(N, comm, restart, iters):
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    dev = BratuDevice(prob, comm)
    u0, y, ut = slab_inputs(dev)
    del ut
    own = dev.slab.own
    rec = {"xnorm2": [], "rsumsq": [], "nfev": []}

    st = dev.backend.zeros(4)

    def cb(x, nfev, cg_iter):
        dev.backend.vec_stats(x.x, st)                         # segment-reduced (rank-count independent)
        rec["xnorm2"].append(float(comm.sum(st[:1])[0]))
        rec["rsumsq"].append(float(x.sumsq))
        rec["nfev"].append(int(nfev))
        log(f"it {len(rec['nfev'])}: nfev {nfev} ||x||^2 {rec['xnorm2'][-1]!r} ||r||^2 {rec['rsumsq'][-1]!r}")

    s = gnk.GNKSolver(prob, y, krylow_restart=restart, max_iter=iters + 1, comm=comm, backend=dev.backend,
                      callback=cb, callback_format="device")
    buf = io.StringIO()
    t0 = time.time()
    with contextlib.redirect_stdout(buf):
        s.setup(u0)
        x0norm = float(s.c[0])                               # ||x_0|| (ref:krylow.py:36)
        del u0
        c0 = dict(comm.counters)
        nsteps = 0
        while not s.step():
            nsteps += 1
        nsteps += 1
        c1 = dict(comm.counters)
        r = s.finish(result_format="torch")
    # collectives and host waits per outer step, the callback's own norm read excluded
    per_step = {k: (c1[k] - c0[k]) / nsteps for k in c0}
    per_step["host_wait"] -= 1.0
    if comm.world > 1:
        per_step["all_gather"] -= 1.0
        per_step["all_gather_bytes"] -= 8.0
    torch.cuda.synchronize()
    out = {"nit": r.nit, "nrev": r.nrev, "njev": r.njev, "success": bool(r.success), "x0norm": x0norm, **rec,
           "k": [t["k"] for t in s.trace], "trials": [t["trials"] for t in s.trace], "stdout": buf.getvalue(),
           "spec": dict(s.spec_stats), "comm_per_step": per_step, "seconds": time.time() - t0}
    del s, r, y, dev, st
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def solve_gn(N, comm, iters, cg_maxiter):
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    dev = BratuDevice(prob, comm)
    u0, y, ut = slab_inputs(dev)
    del ut
    rec = {"xnorm2": [], "rsumsq": [], "nfev": [], "cg_iter": []}

    def cb(x, nfev, cg_iter):
        rec["xnorm2"].append(x.ops.sumsq(x.x))                 # compensated, pairs merged across ranks
        rec["rsumsq"].append(float(x.sumsq))
        rec["nfev"].append(int(nfev))
        rec["cg_iter"].append(int(cg_iter))
        log(f"GN it {len(rec['nfev'])}: cg_iter {cg_iter} nfev {nfev} ||x||^2 {rec['xnorm2'][-1]!r}")

    s = GNSolver(prob, y, max_iter=iters + 1, cg_preconditioner=True, cg_rtol=1e-8, comm=comm,
                 backend=dev.backend, callback=cb, callback_format="device", cg_maxiter=cg_maxiter)
    buf = io.StringIO()
    t0 = time.time()
    c0 = dict(comm.counters)
    with contextlib.redirect_stdout(buf):
        s.setup(u0)
        del u0
        while not s.step():
            pass
        r = s.finish(result_format="torch")
    torch.cuda.synchronize()
    # collectives and host waits of the whole GN solve per CG iteration (the GN outer steps'
    # own residual / Armijo reads included, so an upper bound on the CG iteration's)
    per_cg = {k: (comm.counters[k] - c0[k]) / max(1, s.cg.total_iters) for k in c0}
    out = {"nit": r.nit, "nfev": r.nfev, "njev": r.njev, "success": bool(r.success), **{"it_" + k: v for k, v in rec.items()},
           "t": [t["t"] for t in s.trace], "stdout": buf.getvalue(), "cg_total": s.cg.total_iters,
           "seconds": time.time() - t0, "comm_per_cg_iter": per_cg}
    del s, r, y, dev
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def gn_phase(a, comm, rank, world):
    """GN + CGLS, 8 ranks vs 1 rank (module docstring); returns rank 0's report (None elsewhere)."""
    log(f"multi-rank GN + CGLS, grid {a.grid}, world {world}, CG capped at {a.cg_maxiter}")
    mine = solve_gn(a.grid, comm, a.gn_iters, a.cg_maxiter)
    log(f"multi-rank GN done in {mine['seconds']:.1f} s: cg_iter {mine['it_cg_iter']}")
    every = [None] * world
    dist.all_gather_object(every, mine)
    dist.barrier()
    if rank != 0:
        dist.barrier()
        return None
    try:
        one = solve_gn(a.grid, Comm(single=True, segments=True), a.gn_iters, a.cg_maxiter)
        log(f"single-rank GN done in {one['seconds']:.1f} s")
    except Exception as e:
        log(f"single-rank GN raised {type(e).__name__}: {e}")
        one = {"error": f"{type(e).__name__}: {e}"}
    dist.barrier()
    strip = lambda d: {k: v for k, v in d.items() if k not in ("seconds", "comm_per_cg_iter")}   # noqa: E731
    ranks_identical = all(strip(e) == strip(mine) for e in every)
    exact = ("nit", "nfev", "njev", "success", "it_nfev", "it_cg_iter", "it_xnorm2", "it_rsumsq", "t", "stdout",
             "cg_total")
    bit_identical = all(mine[k] == one.get(k) for k in exact)
    rr = one.get("it_rsumsq", [])
    rel_r = (float(np.max(np.abs(np.sqrt(mine["it_rsumsq"]) - np.sqrt(rr)) / np.sqrt(rr)))
             if len(rr) == len(mine["it_rsumsq"]) and rr else float("inf"))
    ok = bool(ranks_identical and bit_identical and rel_r <= TOL and mine["nit"] == a.gn_iters)
    return {"ok": ok, "ranks_identical": ranks_identical, "bit_identical": bit_identical, "max_rel_rnorm_diff": rel_r,
            "gn_iters": a.gn_iters, "cg_maxiter": a.cg_maxiter, "multi": strip(mine), "single": strip(one),
            "seconds_multi": mine["seconds"], "seconds_single": one.get("seconds"),
            "comm_per_cg_iter_multi": mine["comm_per_cg_iter"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=32768)
    ap.add_argument("--restart", type=int, default=20)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--gn-iters", type=int, default=2)
    ap.add_argument("--cg-maxiter", type=int, default=40)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    log(f"multi-rank solve, grid {a.grid}, world {world}")
    comm = StagedTransportComm()
    mine = solve(a.grid, comm, a.restart, a.iters)
    log(f"multi-rank done in {mine['seconds']:.1f} s: nit {mine['nit']} nrev {mine['nrev']} k {mine['k']}")
    every = [None] * world
    dist.all_gather_object(every, mine)
    dist.barrier()
    if rank != 0:
        dist.barrier()                                      # rank 0's single-rank solve
        if a.gn_iters > 0:
            gn_phase(a, comm, rank, world)
        dist.destroy_process_group()
        return 0
    log("single-rank solve over the whole grid")
    try:
        one = solve(a.grid, Comm(single=True, segments=True), a.restart, a.iters)
        log(f"single-rank done in {one['seconds']:.1f} s")
    except Exception as e:                                   # report it; the other ranks wait at the barrier
        log(f"single-rank solve raised {type(e).__name__}: {e}")
        one = {"error": f"{type(e).__name__}: {e}", "xnorm2": [], "rsumsq": []}
    dist.barrier()
    # traffic counters differ by construction (the edge ranks exchange one halo side): not a decision
    local = ("seconds", "comm_per_step")
    ranks_identical = all({k: v for k, v in e.items() if k not in local} ==
                          {k: v for k, v in mine.items() if k not in local} for e in every)
    keys = ("nit", "nrev", "njev", "success", "nfev", "k", "trials", "stdout")
    same = all(mine[k] == one.get(k) for k in keys)

    def rel(a_, b_):
        a_, b_ = np.sqrt(np.array(a_)), np.sqrt(np.array(b_))
        return np.abs(a_ - b_) / np.abs(b_) if len(a_) == len(b_) and len(b_) else np.array([np.inf])

    ex, er = rel(mine["xnorm2"], one["xnorm2"]), rel(mine["rsumsq"], one["rsumsq"])
    xb = np.maximum(np.maximum(TOL, CANCEL * U * one.get("x0norm", 0.0) / np.sqrt(np.array(one["xnorm2"]))),
                    cycle_spread(len(one["xnorm2"]))) if len(ex) == len(one["xnorm2"]) else np.array([0.0])
    rx, rr = float(np.max(ex)), float(np.max(er))
    bit_identical = bool(mine["xnorm2"] == one.get("xnorm2") and mine["rsumsq"] == one.get("rsumsq"))
    ok = bool(ranks_identical and same and bit_identical)
    rep = {"ok": ok, "grid": a.grid, "world": world, "restart": a.restart, "iters": a.iters,
           "comm_per_step_rank0": mine.get("comm_per_step"),
           "comm_per_step_interior": every[min(1, world - 1)].get("comm_per_step"),
           "ranks_identical": ranks_identical, "bookkeeping_equal": same, "bit_identical": bit_identical,
           "max_rel_xnorm_diff": rx,
           "max_rel_rnorm_diff": rr, "tol": TOL, "rel_xnorm_diff": ex.tolist(), "xnorm_bound": xb.tolist(),
           "x_within_bound": bool(np.all(ex <= xb)) if len(ex) == len(xb) else False, "multi": {k: v for k, v in mine.items() if k != "stdout"},
           "single": {k: v for k, v in one.items() if k != "stdout"}, "shim_calls": dict(comm.staged_calls)}
    if a.gn_iters > 0:
        rep["gn"] = gn_phase(a, comm, rank, world)
        rep["ok"] = bool(rep["ok"] and rep["gn"]["ok"])
        rep["shim_calls_total"] = dict(comm.staged_calls)
    with open(a.out, "w") as f:
        json.dump(rep, f, indent=1)
    log(json.dumps({k: rep[k] for k in ("ok", "ranks_identical", "bookkeeping_equal", "bit_identical",
                                        "max_rel_xnorm_diff", "max_rel_rnorm_diff")}))
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
