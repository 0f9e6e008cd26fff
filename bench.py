#!/usr/bin/env python3
"""Benchmark: GN-Krylov outer iterations/s on the Bratu grid (BASELINE.json metric).

Workload (BASELINE.json configs[1]/metric): Bratu 2-D, ALPHA = 5, LAMBDA = 10,
u0 = u_true + 0.1 N(0, 1) (np.random.seed(42), ref:bratu_pde_test.py:22-36),
fp64, gauss_newton_krylow with krylow_restart = 20 ("Krylov dim 20") on an
N x N interior grid (default N = 8192, the metric's grid).  One *step* = one GNK
outer iteration (LS solve + Armijo trials + basis update); the timed steps cover
a full restart cycle so every basis size 1..21 is represented.

Multi-GPU, one process per GPU: the same grid is row-partitioned over the ranks
(strong scaling); halos + rank-ordered all-gathers over RCCL.  Either launched by
torch.distributed.run (WORLD_SIZE set: every rank checks WORLD_SIZE == --gpus), or
``python bench.py --gpus N`` itself starts the N ranks as child processes with the
same environment torch.distributed.run gives them (``launch_ranks``; the parent never
touches the GPU), relays rank 0's line and fails if any rank fails.  Under RCCL a
box with fewer than N GPUs is refused, never measured as one rank.
value = outer iterations of the whole job per second (max elapsed over ranks).

Also reported: the dominant kernel's roofline (fp64-MFMA Gram pass, HBM-bound,
timed per launch with HIP events over the timed region), the single-vector
JVP microbenchmark (the north star's "8192^2 JVP HBM GB/s"), the whole-step
algorithmic GB/s, and the CPU oracle timed on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import contextlib
import glob
import io
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--repeats", type=int, default=3, help="timed regions of --steps each; value = median")
    ap.add_argument("--grid", type=int, default=8192, help="interior points per side N")
    ap.add_argument("--restart", type=int, default=20)
    ap.add_argument("--version", default="res_old")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU oracle sample budget (0 = skip)")
    ap.add_argument("--jvp-reps", type=int, default=20)
    ap.add_argument("--cg-iters", type=int, default=200, help="CGLS iterations of the C3 line (0 = skip)")
    ap.add_argument("--c5-steps", type=int, default=99,
                    help="capped-C5 line (16384^2, restart 100) outer iterations at N = 1 (0 = skip)")
    ap.add_argument("--no-trial-timer", action="store_true",
                    help="time only the Gram launches in the timed regions (A/B of the trial timer's event cost)")
    ap.add_argument("--segments", choices=("auto", "on", "off"), default="auto",
                    help="rank-count-independent reductions (slab.reduction_segments): auto = on for N > 1")
    return ap.parse_args()


def step_bytes(n, k, a, passes=1.0, fused=False, pending=True):
    """Algorithmic HBM bytes of one outer iteration as implemented, in units of
    8 n bytes (one grid vector); k = Gram columns (settled + the pending one), a = Armijo trials:
      Gram passes              passes * (k + 2)          V (incl. the pending raw g), u, r
      first trial, fused       (k + 3) + [pending]       V -> x; r_old -> g_new; + the w write-back
      first trial, plain       (k + 1) + [pending]       V -> x (+ w write-back)
      other trials             (a - 1) * (k + 1)         basis GEMV
      residual per trial       a * 3                     x, y -> r
      update products          k + 3 unless fused and a = 1   u, r, V -> g (h = V^T g)
    (deferred Gram-Schmidt: no separate CGS or normalisation pass)"""
    first = (k + 3 if fused else k + 1) + (1 if pending else 0)
    trials = first + (a - 1) * (k + 1) + 3 * a
    update = 0 if (fused and a == 1) else k + 3
    return 8.0 * n * (passes * (k + 2) + trials + update)


def cpu_baseline(N, seconds, version, restart, c2_steps=20, grid_c2=1024):
    """The CPU oracle (NumPy restatement of the reference, oracle/) on this host, BASELINE.md's plan:
      * headline: GNK on the same N^2 workload, outer iterations until ``seconds`` of work (setup
        excluded; k = 1..it), with the per-component split (J V products, least squares, Armijo
        trials, basis update);
      * C2: one whole restart cycle (``c2_steps`` iterations, k = 1..20) at 1024^2;
      * the single-vector JVP at N^2 (24 n algorithmic bytes) and the CGLS iteration (Jacobi)."""
    from oracle import gnk_oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    comp = {"jv_products": 0.0, "least_squares": 0.0, "armijo_trials": 0.0, "basis_update": 0.0}
    orig = (O.linear_least_squares, O.armijo_goldstein, O.KrylovBasis.update, O.BratuJacobian.__matmul__)

    def timed(key, fn, pred=None):
        def w(*a, **k):
            t = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                if pred is None or pred(*a):
                    comp[key] += time.perf_counter() - t
        return w

    class Stop(Exception):
        pass

    def run(prob, y, u0, budget_s, max_steps):
        times, t_last = [], [time.perf_counter()]

        def cb(x, nfev, cg_iter):
            now = time.perf_counter()
            times.append(now - t_last[0])
            t_last[0] = now
            if sum(times) >= budget_s or len(times) >= max_steps:
                raise Stop
        t_last[0] = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            try:
                O.gauss_newton_krylow(prob.make_res(y), u0, prob.make_jac(), krylow_restart=restart,
                                      max_iter=10 ** 6, callback=cb, version=version)
            except Stop:
                pass
        return times

    prob, y, u0 = O.bratu_workload(N)
    O.linear_least_squares = timed("least_squares", orig[0])
    O.armijo_goldstein = timed("armijo_trials", orig[1])
    O.KrylovBasis.update = timed("basis_update", orig[2])
    O.BratuJacobian.__matmul__ = timed("jv_products", orig[3], lambda self, V: np.ndim(V) == 2)
    try:
        times = run(prob, y, u0, seconds, 10 ** 6)
    finally:
        O.linear_least_squares, O.armijo_goldstein, O.KrylovBasis.update, O.BratuJacobian.__matmul__ = orig
    it, total = len(times), sum(times)
    comp["other"] = max(total - sum(comp.values()), 0.0)
    out = {"value": it / total, "unit": "outer_iters/s", "cores": threads, "kind": "port",
           "sample": f"oracle/gnk_oracle.py GNK on the same {N}^2 workload, first {it} outer iterations "
                     f"(basis k=1..{it}; {total:.1f} s, setup excluded), OPENBLAS threads={threads}",
           "components_s": {k: round(v, 3) for k, v in comp.items()}}
    # single-vector JVP and one CGLS iteration at N^2 (oracle stencils; A = -J(u0), Jacobi)
    J = prob.make_jac()(u0)
    v = np.random.default_rng(1).standard_normal(N * N)
    jt = []
    for _ in range(3):
        t = time.perf_counter()
        J @ v
        jt.append(time.perf_counter() - t)
    jms = float(np.median(jt))
    out["jvp"] = {"ms": 1e3 * jms, "GBs": 24.0 * N * N / jms / 1e9, "note": "oracle stencil J @ v, 24 n bytes"}
    A = -1 * J
    b = A.T @ prob.make_res(y)(u0)
    dinv = 1 / A.diag_ata()
    ct = []
    O.scipy_cg(lambda p: A.T @ (A @ p), b, psolve=lambda r: dinv * r, rtol=1e-8, maxiter=3,
               callback=lambda x: ct.append(time.perf_counter()))
    out["cg"] = {"ms_per_iter": 1e3 * float(np.mean(np.diff(ct))) if len(ct) > 1 else None,
                 "note": f"oracle scipy-cg recurrence on A^T A at {N}^2, Jacobi, rtol 1e-8"}
    del prob, y, u0, J, v, A, b, dinv
    # C2: one restart cycle at 1024^2, k = 1..20
    p2, y2, u2 = O.bratu_workload(grid_c2)
    t2 = run(p2, y2, u2, 10 ** 9, c2_steps)
    out["c2"] = {"value": len(t2) / sum(t2), "unit": "outer_iters/s", "grid": grid_c2, "steps": len(t2),
                 "sample": f"GNK restart {restart}, the first restart cycle (k = 1..{len(t2)}), setup excluded"}
    return out


CG_BYTES_PER_ITER = 112     # SURVEY §8d model, bytes per unknown: p update 24, J^T J p 24, x/r/z update 64
CG_BYTES_MOVED = 96         # what the fused iteration moves: step matvec 56 (d, z, p, x in; p', q, x out)
                            # + r / z update 40 (q, r, dinv in; r, z out)


def gn_cg_line(args, prob, u0, y, comm, device, world, backend):
    """CGLS of the first Gauss-Newton step (A = -J(u0), right-hand side res(u0),
    ref:gauss_newton.py:112-114) at cg_rtol = 1e-8 (Jacobi preconditioner, :50-58), capped at
    --cg-iters iterations (a full solve at 8192^2 takes far more).  Reports CG iterations/s of the
    whole job and the fused J^T J p kernel's per-launch rate."""
    from gauss_newton_via_generalized_krylov_subspaces_amd import _native
    from gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton import BratuGNOps, DeviceCG
    N = args.grid
    n = N * N
    ops = BratuGNOps(prob, y, comm, device, backend)
    cg = DeviceCG(ops)
    u = ops.load(u0)
    r0 = ops.vec()
    ops.residual(u, r0)                                                        # res(u0)
    comm.halo(r0, N, ops.dev.slab.nrows)
    be = ops.be
    cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=5)             # warm-up
    cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=5, variant="single_reduction")
    cap = args.cg_iters + 8
    be.timer_start(_native.TIMER_CG_MATVEC, cap)
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, iters = cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=args.cg_iters)
    torch.cuda.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    ml = be.timer_collect(cap)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # the single-reduction recurrence (SURVEY f2 option): one host read per CG iteration instead of two
    comm.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    _, iters_sr = cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=args.cg_iters,
                           variant="single_reduction")
    torch.cuda.synchronize()
    comm.barrier()
    el_sr = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([el_sr], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el_sr = t.item()
    # the iteration's split: every CG kernel class timed per launch (event pairs around each), in a solve of
    # its own so the timed solve above keeps one event pair per iteration
    cap6 = 6 * (args.cg_iters + 8)
    be.timer_start(_native.TIMER_CG_MATVEC, cap6)
    be.timer_add(_native.TIMER_CG_XR)
    be.timer_add(_native.TIMER_CG_AUX)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    _, iters_split = cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=args.cg_iters)
    torch.cuda.synchronize()
    el_split = time.perf_counter() - t2
    sl_ = be.timer_collect_ids(cap6)
    split = {}
    for name, tid in (("matvec", _native.TIMER_CG_MATVEC), ("xr", _native.TIMER_CG_XR), ("aux", _native.TIMER_CG_AUX)):
        got = [(m, b) for i, m, b in sl_ if i == tid]
        tot = sum(m for m, _ in got)
        split[name] = {"launches": len(got), "ms_per_iter": tot / max(iters_split, 1),
                       "avg_launch_ms": tot / max(len(got), 1)}
        if name != "aux" and got:
            by = float(np.mean([b for _, b in got]))
            split[name]["algorithmic_bytes_per_launch"] = by
            split[name]["GBs"] = by / (split[name]["avg_launch_ms"] * 1e-3) / 1e9
    busy = sum(v["ms_per_iter"] for v in split.values())
    split["wall_ms_per_iter"] = 1e3 * el_split / max(iters_split, 1)
    split["gaps_ms_per_iter"] = split["wall_ms_per_iter"] - busy
    split["note"] = ("every CG launch bracketed by HIP events (a separate solve): matvec = k_cg_matvec_m, xr = k_cg_xr, "
                     "aux = the partial-sum reductions and k_cg_scalars; gaps = wall - kernels (launch gaps, the "
                     "lagged host read)")
    m_ms = float(np.mean([m for m, _ in ml])) if ml else float("nan")
    m_by = float(np.mean([b for _, b in ml])) if ml else float("nan")
    m_gbs = m_by / (m_ms * 1e-3) / 1e9 if ml else float("nan")
    return {"workload": f"bratu_{N}x{N}_gn_cgls_rtol1e-8_first_step", "cg_iters": iters,
            "value": iters / elapsed, "unit": "cg_iters/s", "ms_per_iter": 1e3 * elapsed / max(iters, 1),
            "algorithmic_GBs": CG_BYTES_PER_ITER * n * iters / elapsed / 1e9,
            "bytes_per_iter": CG_BYTES_PER_ITER * n,
            "bytes_per_iter_moved": CG_BYTES_MOVED * n,
            "moved_GBs": CG_BYTES_MOVED * n * iters / elapsed / 1e9,
            "split": split,
            "single_reduction": {"cg_iters": iters_sr, "value": iters_sr / el_sr, "unit": "cg_iters/s",
                                 "ms_per_iter": 1e3 * el_sr / max(iters_sr, 1),
                                 "note": "cg_variant='single_reduction' (Chronopoulos-Gear, non-parity option): "
                                         "one host read per iteration, 120 n bytes"},
            "note": "timed: one CGLS solve capped at cg_iters (b = A^T y, Jacobi diag and the initial update "
                    "included); scipy's 10 n cap would need millions of iterations at rtol 1e-8",
            "matvec": {"kernel": "k_cg_matvec_m (p = z + beta p, lagged x += alpha p, q = J^T J p, 13-point, "
                                 "row marching)", "avg_launch_ms": m_ms,
                       "GBs": m_gbs, "frac_of_peak": m_gbs / HBM_PEAK_GBS,
                       "algorithmic_bytes_per_launch": m_by}}


FP64_MFMA_PEAK_TFS = 78.6   # MI355X fp64 matrix peak (the MFMA probe measures 72 TF/s)


def gram_useful_flops(n, k):
    """Useful fp64 flops of one Gram pass over [J V T | r] (k basis columns, n points): the triangular
    transform W = (J V) T (k (k + 1) per point) and the symmetric Gram of the k + 1 columns
    ((k + 1) (k + 2) per point, one triangle)."""
    return float(n) * (k * (k + 1) + (k + 1) * (k + 2))


def c5_capped_line(args, comm, device, grid=16384, restart=100):
    """SURVEY §8d C5 with k capped (16384^2, Krylov dim 100; k = 200 needs 429 GB, more than one GPU holds):
    one whole restart cycle after one warm-up step -- basis sizes k = 2..100 -- timed as one region, with every
    Gram pass timed per launch (HIP events): outer it/s, the Gram pass by k, and its fp64-MFMA fraction
    (useful flops / time / peak) -- the wide-basis MFMA path of ref:krylow.py:72-73 / gauss_newton_krylow.py:81-82."""
    import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
    from gauss_newton_via_generalized_krylov_subspaces_amd import _native
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs
    prob = gnk.BratuPdeProblem(grid + 1, 5, 10)
    stage = BratuDevice(prob, comm, device)
    u0, y, _ = slab_inputs(stage)
    s = gnk.GNKSolver(prob, y, krylow_restart=restart, tol=1e-8, max_iter=10 ** 9, version=args.version,
                      comm=comm, device=device, backend=stage.backend)
    s.setup(u0)
    be = s.be
    steps = min(args.c5_steps, restart - 1)
    with contextlib.redirect_stdout(io.StringIO()):
        s.step()                                                   # warm-up: k = 1
        cap = 8 * (steps + 2)
        be.timer_start(_native.TIMER_GRAM, cap)
        be.timer_add(_native.TIMER_TRIAL)
        tr0 = len(s.trace)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            if s.step():
                break
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    got = be.timer_collect_ids(cap)
    done = len(s.trace) - tr0
    n = s.dev.slab.nrows * grid
    trials = [(m, b) for i, m, b in got if i == _native.TIMER_TRIAL]
    got = [(i, m, b) for i, m, b in got if i == _native.TIMER_GRAM]
    by_k, flops, gms = {}, 0.0, 0.0
    for _, m, b in got:
        kk = int(round(b / (8.0 * n))) - 2
        by_k.setdefault(kk, []).append(m)
        flops += gram_useful_flops(n, kk)
        gms += m
    tr = s.trace[tr0:]
    del s, stage, u0, y
    torch.cuda.empty_cache()
    tfs = flops / (gms * 1e-3) / 1e12 if gms else float("nan")
    return {"workload": f"bratu_{grid}x{grid}_gnk_krylov_dim{restart}_capped", "value": done / el,
            "unit": "outer_iters/s", "steps": done, "ms_per_step": 1e3 * el / max(done, 1),
            "basis_k_range": [min(t["k"] for t in tr), max(t["k"] for t in tr)] if tr else None,
            "armijo_trials": int(sum(t["trials"] for t in tr)),
            "gram": {"share_of_step_time": gms * 1e-3 / el, "launches": len(got), "useful_TFLOPs": tfs,
                     "fp64_mfma_frac": tfs / FP64_MFMA_PEAK_TFS, "peak_TFLOPs": FP64_MFMA_PEAK_TFS,
                     "flops_model": "n [k (k + 1) + (k + 1) (k + 2)] per pass (triangular transform + one Gram "
                                    "triangle of k + 1 columns)",
                     "by_k": {str(kk): {"ms": float(np.mean(v)),
                                        "GBs": 8.0 * n * (kk + 2) / (np.mean(v) * 1e-3) / 1e9,
                                        "TFLOPs": gram_useful_flops(n, kk) / (np.mean(v) * 1e-3) / 1e12}
                              for kk, v in sorted(by_k.items())}},
            "trial": {"kernel": "first Armijo trial + update products: k_gemv_vjpg (<= 24 columns), k_trial_w (25..208, "
                                "LDS tiles)", "launches": len(trials),
                      "share_of_step_time": sum(m for m, _ in trials) * 1e-3 / el,
                      "by_vectors": {str(v): {"ms": float(np.mean([m for m, b in trials if int(round(b / (8.0 * n))) == v])),
                                              "GBs": 8.0 * n * v / (np.mean([m for m, b in trials
                                                                             if int(round(b / (8.0 * n))) == v]) * 1e-3) / 1e9}
                                     for v in sorted({int(round(b / (8.0 * n))) for _, b in trials})}},
            "note": "C5 at 16384^2 with the basis capped at 100 columns (restart 100): V = 101 x 2.15 GB; the literal "
                    "k = 200 (429 GB) does not fit one GPU. One warm-up step (k = 1), then the cycle's steps timed."}


def prewarm(args, comm, device):
    """HIP loads a kernel's code object at its first launch (~1 ms each).  One restart cycle on a
    256^2 grid (same dispatch: N % 128 == 0, same k range and version) makes every kernel variant
    of the timed steps resident before the clock starts."""
    import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs
    prob = gnk.BratuPdeProblem(256 + 1, 5, 10)
    stage = BratuDevice(prob, comm, device)
    u0, y, _ = slab_inputs(stage)
    s = gnk.GNKSolver(prob, y, krylow_restart=args.restart, tol=1e-8, max_iter=10 ** 9, version=args.version,
                      comm=comm, device=device, backend=stage.backend)
    s.setup(u0)
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(args.restart + 2):
            if s.step():
                break
    torch.cuda.synchronize()


def c2_gpu(args, comm, device, grid=1024):
    """GPU outer iterations/s on C2 (1024^2, restart 20): the second restart cycle after setup (the
    first warms the kernels), for the like-for-like comparison with the CPU's C2 cycle."""
    import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs
    prob = gnk.BratuPdeProblem(grid + 1, 5, 10)
    stage = BratuDevice(prob, comm, device)
    u0, y, _ = slab_inputs(stage)
    s = gnk.GNKSolver(prob, y, krylow_restart=args.restart, tol=1e-8, max_iter=10 ** 9, version=args.version,
                      comm=comm, device=device, backend=stage.backend)
    s.setup(u0)
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(args.restart):
            s.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.restart):
            s.step()
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return {"value": args.restart / el, "unit": "outer_iters/s", "steps": args.restart,
            "note": "GPU, second restart cycle (k = 1..20) of the same C2 run"}


def pmc_traffic(config_key, window, section=None):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (tools/pmc_summary.py) of this
    configuration AND this timed window: same warmup / steps / repeats / launch count and the same
    algorithmic bytes per launch (so the same basis sizes).  section None: the Gram pass; "trial": the
    first-trial kernel.  Otherwise (None, None): the line reports traffic null."""
    count = "trial_launches" if section == "trial" else "gram_launches"
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("config") != config_key:
            continue
        if section:
            d = d.get(section) or {}
        w = d.get("window") or {}
        if (d.get("traffic_bytes_per_launch")
                and all(w.get(k) == window[k] for k in ("warmup", "steps", "repeats", count))
                and abs(w.get("algorithmic_bytes_per_launch", 0.0) - window["algorithmic_bytes_per_launch"])
                <= 1e-9 * window["algorithmic_bytes_per_launch"]):
            return d["traffic_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def pmc_sq(config_key, window):
    """fp64 pipe use of the Gram passes from a committed SQ counter summary (tools/pmc_bench_sq.sh ->
    tools/pmc_sq_summary.py) of this configuration and this timed window (same warmup / steps / repeats /
    launch count / algorithmic bytes per launch): the window's mfma_busy (MFMA pipe cycles / SIMD cycles)
    and per basis size k (mfma_busy, share of wave time waiting on operands, wave instructions).  The
    last matching summary in path order wins; (None, None) when none matches."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_sq_summary*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        w = d.get("window") or {}
        if (d.get("config") == config_key and d.get("mfma_busy") is not None
                and all(w.get(k) == window[k] for k in ("warmup", "steps", "repeats", "gram_launches"))
                and abs(w.get("algorithmic_bytes_per_launch", 0.0) - window["algorithmic_bytes_per_launch"])
                <= 1e-9 * window["algorithmic_bytes_per_launch"]):
            per_k = {k: {"kernel": v["kernel"], "mfma_busy": v["mfma_busy"], "wait_inst_any_frac": v["wait_inst_any_frac"],
                         "valu_per_launch": v["insts_valu"], "mfma_per_launch": v["insts_mfma"]}
                     for k, v in d["per_k"].items()}
            return {"mfma_busy": d["mfma_busy"], "by_k": per_k}, os.path.relpath(path, ROOT)
    return None, None


def stream_floor(be, n, device, reps):
    """Measured HBM streaming floor on this box (gnk_probe_stream, HIP events): triad a = b + s c
    (24 n bytes), read-only (8 n) and copy (16 n) over n doubles, the median of reps launches each --
    what a perfectly coalesced kernel of that access mix reaches, the yardstick for the HBM-bound
    kernels beside the 8 TB/s spec peak."""
    from gauss_newton_via_generalized_krylov_subspaces_amd import _native
    a = torch.empty(n, dtype=torch.float64, device=device)
    b = torch.ones(n, dtype=torch.float64, device=device)
    c = torch.ones(n, dtype=torch.float64, device=device)
    out = {}
    for name, mode in (("triad", 0), ("read", 1), ("copy", 2)):
        for _ in range(3):
            be.probe_stream(a, b, c, 0.5, n, mode)
        be.timer_start(_native.TIMER_PROBE, reps)
        for _ in range(reps):
            be.probe_stream(a, b, c, 0.5, n, mode)
        got = be.timer_collect(reps)
        ms = float(np.median([m for m, _ in got]))
        out[name] = {"ms": ms, "GBs": got[0][1] / (ms * 1e-3) / 1e9, "bytes": got[0][1]}
    del a, b, c
    out["kernel"] = "k_probe_stream (16-B accesses, 4 in flight per lane, one pass over n doubles)"
    return out


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, cmd, env=None, poll_s=0.2, grace_s=15.0):
    """Start ``cmd`` as ranks 0..n-1 of one single-node job (the variables torch.distributed.run sets:
    RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, GROUP_RANK, MASTER_ADDR = 127.0.0.1, a free
    MASTER_PORT), each in a process group of its own, and wait.  The ranks inherit stdout / stderr (rank 0
    prints the result line).  If any rank exits non-zero the others are terminated (then killed after
    ``grace_s``) and that exit code is returned; 0 when all succeed.  Child processes, never exec: the
    caller must not have initialised the GPU."""
    import signal
    import subprocess
    base = dict(os.environ if env is None else env)
    base.update(WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = []

    def _forward(signum, frame):                 # the driver's timeout / Ctrl-C reaches every rank's group
        for p in procs:
            with contextlib.suppress(ProcessLookupError):
                os.killpg(p.pid, signum)
        raise SystemExit(128 + signum)

    old_handlers = {sig: signal.signal(sig, _forward) for sig in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)}
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(cmd, env=e, start_new_session=True))
    failed = 0
    try:
        while [p.poll() for p in procs].count(None):          # poll every rank (no short-circuit)
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                failed = bad[0]
                break
            time.sleep(poll_s)
        else:
            bad = [p.returncode for p in procs if p.returncode != 0]
            failed = bad[0] if bad else 0
    finally:
        live = [p for p in procs if p.poll() is None]
        for sig in (signal.SIGTERM, signal.SIGKILL):
            for p in live:
                with contextlib.suppress(ProcessLookupError):
                    os.killpg(p.pid, sig)
            t_end = time.time() + grace_s
            while live and time.time() < t_end:
                live = [p for p in live if p.poll() is None]
                time.sleep(poll_s)
            if not live:
                break
        for p in procs:
            with contextlib.suppress(Exception):
                p.wait(timeout=grace_s)
        for sig, h in old_handlers.items():
            signal.signal(sig, h)
    return failed if failed >= 0 else 1            # a rank killed by a signal: 1


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    backend = os.environ.get("GNK_BENCH_BACKEND", "nccl")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N`: start the N ranks here (this process has not touched the GPU;
        # device_count does not initialise it on this image)
        if backend != "gloo" and torch.cuda.device_count() < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs under RCCL, "
                             f"this node has {torch.cuda.device_count()}; refusing to measure fewer ranks")
        sys.exit(launch_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing a mislabelled run")
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        # GNK_BENCH_BACKEND=gloo: rehearsal of the multi-rank bench on fewer GPUs than ranks (ranks
        # share cards, collectives staged through the host); the measured runs use RCCL, one GPU each
        if backend == "gloo":
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group("gloo")
        else:
            if torch.cuda.device_count() < world:
                raise SystemExit(f"bench.py: rank {rank}: {world} ranks under RCCL need {world} GPUs, "
                                 f"this node has {torch.cuda.device_count()}")
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    else:
        torch.cuda.set_device(0)
    device = torch.device("cuda", torch.cuda.current_device())

    import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
    from gauss_newton_via_generalized_krylov_subspaces_amd import _native
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm

    N = args.grid
    n = N * N
    comm = Comm(segments={"auto": None, "on": True, "off": False}[args.segments])
    prewarm(args, comm, device)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    # this rank's slabs of u0 and y = F(u_true) (ref:bratu_pde_test.py:22-36), built per rank: no
    # whole-grid vector on any host or GPU (inputs.py)
    stage = BratuDevice(prob, comm, device)
    u0, y, _ = slab_inputs(stage)
    solver = gnk.GNKSolver(prob, y, krylow_restart=args.restart, tol=1e-8, max_iter=10 ** 9,
                           version=args.version, comm=comm, device=device, backend=stage.backend)
    solver.setup(u0)
    be = solver.be
    warm_s = []                 # per-step times of the warm-up steps (k = 1..warmup), synchronised each
    # the warm-up's launches are counted (not timed into the result) so the PMC / trace tools can find
    # the timed regions' launches of each kernel class among all bench-grid launches
    wcap = 8 * (args.warmup + 1)
    be.timer_start(_native.TIMER_GRAM, wcap)
    be.timer_add(_native.TIMER_TRIAL)
    with contextlib.redirect_stdout(io.StringIO()):
        for _ in range(args.warmup):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            solver.step()
            torch.cuda.synchronize()
            warm_s.append(time.perf_counter() - t0)
    wl = be.timer_collect_ids(wcap)
    gram_offset = sum(1 for i, _, _ in wl if i == _native.TIMER_GRAM)    # bench-grid launches before the
    trial_offset = sum(1 for i, _, _ in wl if i == _native.TIMER_TRIAL)  # first timed region
    # --repeats timed regions of exactly --steps outer iterations each (with the default 20 steps one
    # region is one whole restart cycle, k = 1..20); value = the median region's rate
    cap = 8 * (args.steps + 1)
    k_trace0 = len(solver.trace)
    passes0 = solver.lls.passes
    regions, launches, tlaunches = [], [], []
    comm0 = dict(comm.counters)
    fb0 = be.segment_fallbacks()
    for _ in range(args.repeats):
        be.timer_start(_native.TIMER_GRAM, cap)
        if not args.no_trial_timer:
            be.timer_add(_native.TIMER_TRIAL)
        tr0 = len(solver.trace)
        comm.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            for _ in range(args.steps):
                if solver.step():
                    break
        torch.cuda.synchronize()
        comm.barrier()
        el = time.perf_counter() - t0
        got = be.timer_collect_ids(cap)
        launches += [(m, b) for i, m, b in got if i == _native.TIMER_GRAM]
        tlaunches += [(m, b) for i, m, b in got if i == _native.TIMER_TRIAL]
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = t.item()
        regions.append((len(solver.trace) - tr0, el))
    fallbacks = be.segment_fallbacks() - fb0            # the timed steps' unsegmented reductions only
    comm_steps = max(1, sum(st for st, _ in regions))
    comm_per_step = {key: (comm.counters[key] - comm0[key]) / comm_steps for key in comm0}
    rates = [st / el for st, el in regions]
    imed = int(np.argsort(rates)[len(rates) // 2])
    steps_done, elapsed = regions[imed]
    elapsed_all = sum(el for _, el in regions)

    # whole-step algorithmic bytes (global grid) over all timed steps
    tr = solver.trace[k_trace0:]
    passes = solver.lls.passes - passes0
    ppi = passes / max(len(tr), 1)
    fuse_ok = args.version == "res_old"
    total_bytes = sum(step_bytes(n, s["k"], s["trials"], ppi, fused=fuse_ok and s["k"] <= solver.basis.FUSE_KMAX,
                                 pending=s["k"] > 1)
                      for s in tr)
    # dominant kernel: Gram pass (per-launch events; bytes are this rank's slab)
    g_ms = [m for m, _ in launches]
    g_by = [b for _, b in launches]
    g_avg_ms = float(np.mean(g_ms)) if g_ms else float("nan")
    g_avg_bytes = float(np.mean(g_by)) if g_by else float("nan")
    g_gbs = g_avg_bytes / (g_avg_ms * 1e-3) / 1e9 if g_ms else float("nan")
    window = {"warmup": args.warmup, "steps": args.steps, "repeats": args.repeats, "gram_launch_offset": gram_offset,
              "gram_launches": len(g_ms), "algorithmic_bytes_per_launch": g_avg_bytes}
    # the first Armijo trial + update products (k_gemv_vjpg), the largest kernel by time
    t_ms = [m for m, _ in tlaunches]
    t_by = [b for _, b in tlaunches]
    t_avg_ms = float(np.mean(t_ms)) if t_ms else float("nan")
    t_avg_bytes = float(np.mean(t_by)) if t_by else float("nan")
    t_gbs = t_avg_bytes / (t_avg_ms * 1e-3) / 1e9 if t_ms else float("nan")
    twindow = {"warmup": args.warmup, "steps": args.steps, "repeats": args.repeats,
               "trial_launch_offset": trial_offset, "trial_launches": len(t_ms),
               "algorithmic_bytes_per_launch": t_avg_bytes}
    if os.environ.get("GNK_BENCH_WINDOW_OUT") and rank == 0:
        # the Gram and first-trial launches of the timed regions, for tools/pmc_summary.py and
        # tools/rocprof_window.py (they run this same command under rocprofv3 and keep exactly these)
        with open(os.environ["GNK_BENCH_WINDOW_OUT"], "w") as f:
            json.dump({**window, "grid": N, "launch_bytes": g_by,
                       "trial": {**twindow, "launch_bytes": t_by}}, f)
    gram_share = sum(g_ms) * 1e-3 / elapsed_all if g_ms else float("nan")
    # per basis size: columns = bytes / (8 n_rank) - 2 (V, u, r); kernel as gnk_gram dispatches a pass
    # with P^-1 and r: VALU k <= 7, staged on 4x4x4 blocks k = 8..31 (N % 128 == 0; else VALU one point per lane
    # at 8, 9), chunked
    # k_gram_w up to 31 columns (+ r), the marching k_gram_x for 3..7 column blocks (N % 32 == 0; else the
    # chunked k_gram_w at 3 blocks and the prefetching k_gram_wp at 4), the pair-split k_gram beyond
    def gram_kernel(kk):
        if kk <= 7:
            return "k_gram_v"
        if kk <= 31 and N % 128 == 0:
            return "k_gram_q"                  # the 4x4x4-block staged pass (k_gram_s / k_gram_w with GNK_TUNE_GRAM_Q 1)
        if kk <= 9:
            return "k_gram_v1"
        if kk + 1 <= 32:
            return "k_gram_w"
        if (kk + 16) // 16 <= 7 and N % 32 == 0:
            return "k_gram_x"
        return "k_gram_w" if kk + 1 <= 48 else "k_gram_wp" if kk + 1 <= 64 else "k_gram"

    n_rank = solver.dev.slab.nrows * N
    by_k = {}
    for m, b in launches:
        kk = int(round(b / (8.0 * n_rank))) - 2
        by_k.setdefault(kk, []).append(m)
    gram_by_k = {str(kk): {"ms": float(np.mean(v)), "GBs": 8.0 * n_rank * (kk + 2) / (np.mean(v) * 1e-3) / 1e9,
                           "kernel": gram_kernel(kk)} for kk, v in sorted(by_k.items())}

    # JVP microbenchmark (single vector, 24 n bytes per launch)
    sl = solver.dev.slab
    v = solver.dev.vec()
    out = solver.dev.vec()
    gen = torch.Generator(device=device).manual_seed(1)
    v[sl.own] = torch.randn(sl.nrows * N, generator=gen, device=device, dtype=torch.float64)
    uu = solver.xb[solver.uJ]
    for _ in range(3):
        be.jvp(uu, v, out)
    be.timer_start(_native.TIMER_JVP, args.jvp_reps)
    for _ in range(args.jvp_reps):
        be.jvp(uu, v, out)
    jl = be.timer_collect(args.jvp_reps)
    j_ms = float(np.median([m for m, _ in jl]))
    j_gbs = jl[0][1] / (j_ms * 1e-3) / 1e9
    stream = stream_floor(be, n_rank, device, args.jvp_reps)
    trial_by_k = {}
    for m, b in tlaunches:
        trial_by_k.setdefault(int(round(b / (8.0 * n_rank))), []).append(m)

    spec_stats = dict(solver.spec_stats)
    del solver, v, out, uu                      # free the GNK state (the basis) before the CG line
    torch.cuda.empty_cache()
    cg_line = gn_cg_line(args, prob, u0, y, comm, device, world, stage.backend) if args.cg_iters > 0 else None

    c5_line = None
    if world == 1 and args.c5_steps > 0:
        torch.cuda.empty_cache()
        c5_line = c5_capped_line(args, comm, device)
    config_key = f"bratu{N}_gnk_restart{args.restart}_{args.version}_ranks{world}"
    traffic, traffic_src = pmc_traffic(config_key, window)
    t_traffic, t_traffic_src = pmc_traffic(config_key, twindow, section="trial")
    sq, sq_src = pmc_sq(config_key, window)
    result = {
        "metric": "GN-Krylov outer iters/sec + JVP HBM GB/s, Bratu 8192² fp64, 1/2/4/8 GPUs",
        "value": steps_done / elapsed,
        "unit": "outer_iters/s",
        "n_gpus": world,
        "steps": steps_done,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / max(steps_done, 1),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Bratu u_true + 0.1 N(0,1), seed 42; ref:bratu_pde_test.py:22-36)",
        "config": {"workload": f"bratu_{N}x{N}_gnk_krylov_dim{args.restart}", "grid": N, "unknowns": n,
                   "krylow_restart": args.restart, "version": args.version, "ALPHA": 5, "LAMBDA": 10,
                   "basis_k_range": [min(s["k"] for s in tr), max(s["k"] for s in tr)] if tr else None,
                   "armijo_trials": int(sum(s["trials"] for s in tr)),
                   "parallelism": f"slab{world}",
                   "transport": (dist.get_backend() if world > 1 else "none"),
                   "reduction_segments": int(stage.seg_rows),
                   # reductions of the timed steps that ran unsegmented while segments were on (wide Gram
                   # passes): 0 = the timed steps' bits do not depend on the rank count
                   "segment_fallbacks": int(fallbacks)},
        "roofline": {"kernel": "Gram pass of the CholeskyQR solve, J V T on the fly (k_gram_v: VALU, k <= 7; "
                               "k_gram_q: staged, 4x4x4 fp64 MFMA blocks, k >= 8)", "bound": "hbm",
                     "achieved": g_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": g_gbs / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_over_algorithmic": (traffic / g_avg_bytes) if traffic else None, "window": window,
                     "avg_launch_ms": g_avg_ms, "algorithmic_bytes_per_launch": g_avg_bytes,
                     "launches": len(g_ms), "share_of_step_time": gram_share, "by_k": gram_by_k,
                     "mfma_busy": sq["mfma_busy"] if sq else None, "mfma_busy_source": sq_src,
                     "mfma_busy_by_k": sq["by_k"] if sq else None,
                     "mfma_busy_note": "SQ_VALU_MFMA_BUSY_CYCLES / (128 GRBM_GUI_ACTIVE) over the window's Gram "
                                       "launches (tools/pmc_bench_sq.sh; f64 MFMA = 64 busy cycles each)",
                     "trial": {"kernel": "k_gemv_vjpg (first Armijo trial x = V c, g = -J(x)^T r_old, h = V^T g; "
                                         "pending column w = g - V hh materialised), one launch per step",
                               "bound": "hbm", "achieved": t_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": t_gbs / HBM_PEAK_GBS, "traffic": t_traffic, "traffic_source": t_traffic_src,
                               "traffic_over_algorithmic": (t_traffic / t_avg_bytes) if t_traffic else None,
                               "avg_launch_ms": t_avg_ms, "algorithmic_bytes_per_launch": t_avg_bytes,
                               "bytes_model": "8 n (k + 3 + 2 [pending]): k settled columns, r in, x, g out, w r/w",
                               "launches": len(t_ms), "window": twindow,
                               "share_of_step_time": sum(t_ms) * 1e-3 / elapsed_all if t_ms else None,
                               "frac_of_stream_floor": {m: t_gbs / stream[m]["GBs"] for m in ("read", "triad")},
                               "by_vectors": {str(kk): {"ms": float(np.mean(v)),
                                                        "GBs": 8.0 * n_rank * kk / (np.mean(v) * 1e-3) / 1e9}
                                              for kk, v in sorted(trial_by_k.items())}}},
        "stream_floor": stream,
        "jvp": {"kernel": "k_jvp (J(u) v, 5-point stencil)", "grid": N, "median_ms": j_ms, "GBs": j_gbs,
                "frac_of_peak": j_gbs / HBM_PEAK_GBS, "algorithmic_bytes": jl[0][1]},
        "repeats": [{"steps": st, "seconds": el, "outer_iters_per_s": st / el} for st, el in regions],
        "step_algorithmic_GBs": total_bytes / elapsed_all / 1e9,
        "gram_passes_per_step": ppi,
        "comm_per_step": comm_per_step,
        "speculated_solves": spec_stats,
    }
    if cg_line is not None:
        result["gn_cg"] = cg_line
    if c5_line is not None:
        result["c5_capped"] = c5_line
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        try:
            cb_ = cpu_baseline(N, args.cpu_seconds, args.version, args.restart)
            # the GPU on the CPU sample's own windows: the first outer iterations of this workload
            # (the warm-up steps, k = 1..) and the C2 restart cycle at 1024^2
            kk = min(len(warm_s), int(cb_["sample"].split("first ")[1].split(" ")[0]))
            if kk:
                cb_["gpu_same_window"] = {"value": kk / sum(warm_s[:kk]), "unit": "outer_iters/s", "steps": kk,
                                          "note": "GPU, first steps of the same workload, each synchronised"}
            cb_["c2"]["gpu"] = c2_gpu(args, comm, device)
            result["cpu_baseline"] = cb_
        except Exception as e:  # report, never hide
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
