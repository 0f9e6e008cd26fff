"""Multi-slab run of the HIP path on ONE GPU (all ranks on cuda:0; gloo with host-staged
collectives -- RCCL refuses two ranks on one device).  Exercises what single-rank runs cannot:
slabs with row0 > 0, halo-filled ghost rows, rank-ordered reductions feeding the HIP kernels
(Gram, fused first trial, CGS, CG), and the per-rank input staging of inputs.py.

  python -m torch.distributed.run --standalone --nproc-per-node W tests/multislab_worker.py \\
      --grid N --out result.json

Driven by tests/test_gpu_multislab.py.  Every rank runs every case; rank 0 collects all ranks'
results, repeats each solve single-rank and writes the comparison to --out:
  * all ranks took identical decisions (bookkeeping, stdout, per-iteration nfev) and hold the same
    iterate norms bit for bit;
  * multi-rank vs single-rank: bookkeeping identical; where the world divides 8 and N % 8 == 0 the
    reductions are segmented (slab.reduction_segments, gnk_set_segments: on by default for several
    ranks, asked for on the single rank) and every per-iteration ||x_k|| and the final x must agree BIT
    FOR BIT, GNK and GN alike; otherwise (world 3) within the case's bound: GN + CGLS at north_star's
    1e-10 (the CG scalars are compensated pairs merged across ranks, slab.Comm.sum_pairs), GNK at the
    spread of the reference's own arithmetic reordered as 2 .. 8 slabs order it
    (tests/test_oracle_sensitivity.py);
  * multi-rank vs the ORACLE (oracle/gnk_oracle.py, on rank 0's host): GNK bookkeeping and stdout
    identical, ||x_k|| within the same sensitivity bound; GN against the oracle with exactly rounded
    CG dot products (math.fsum -- what the device's compensated sums compute): bookkeeping and every
    cg_iter identical, ||x_k|| within the reordered-CG-dot spread (oracle_bound);
  * ``--transport shim``: slab.Comm's RCCL branches (device all-gathers, pinned read_async, k_rank_sum,
    sum_device, device halos) with the bytes moved over gloo underneath (tests/transport_shim.py);
  * GNKSolver on slab-staged inputs (u0, y built per rank, no full-grid vector) == the same solver
    on full-grid host inputs, bit for bit.
"""
import argparse
import contextlib
import io
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm, reduction_segments  # noqa: E402

# ||x_k|| bound, multi-rank vs single-rank (every reduction summed in a different order): GNK at
# max(1e-10, the spread of the reference's own arithmetic reordered as 2 .. 8 slabs order it, permuted
# QR, exact k = 1 sums, 1 vs 8 BLAS threads -- tests/tolerances.py, cases multislab<grid>_<version>);
# GN + CGLS at max(1e-10, the spread of the reference's GN with its CG dot products summed in other
# orders -- pairwise, reversed, 2 .. 8 slab blocks, 8 BLAS threads: cases gn<grid>[_pre]).
def bound(kind, kw, grid):
    """multi-rank vs one rank: GN + CGLS carries the compensated CG sums across ranks, so north_star's
    1e-10 (measured: bit-identical); GNK the slab-reordering spread of the reference's arithmetic."""
    from tests import tolerances as T
    if kind == "gnk":
        return T.trajectory_bound(f"multislab{grid}_{kw['version']}")
    return T.NORTH_STAR


def oracle_bound(kind, kw, grid):
    """vs the oracle: GNK as above; GN + CGLS against the exactly-rounded-dot oracle at the spread of the
    reference's GN under reordered CG dot products (cases gn<grid>[_pre]): the device's fused 13-point
    J^T J p and its x / r updates round differently from the oracle's two passes, and ~115 Jacobi CG
    iterations per step carry that difference (measured 3.6e-10 .. 8.2e-10 at grids 384 / 256)."""
    from tests import tolerances as T
    if kind == "gnk":
        return T.trajectory_bound(f"multislab{grid}_{kw['version']}")
    return T.trajectory_bound(f"gn{grid}" + ("_pre" if kw.get("cg_preconditioner") else ""))


def exact_cg(matvec, b, psolve=None, rtol=1e-5, maxiter=None, callback=None):
    """oracle.scipy_cg (scipy iterative.py:305-422) with every dot product exactly rounded (math.fsum)."""
    import math
    dot = lambda a, c: math.fsum(a * c)                     # noqa: E731
    bnrm2 = math.sqrt(dot(b, b))
    atol = max(0.0, float(rtol) * float(bnrm2))
    if bnrm2 == 0:
        return b, 0
    maxiter = len(b) * 10 if maxiter is None else maxiter
    x, r, rho_prev, p = np.zeros_like(b), b.copy(), None, None
    for it in range(maxiter):
        if math.sqrt(dot(r, r)) < atol:
            return x, 0
        z = r if psolve is None else psolve(r)
        rho = dot(r, z)
        if it > 0:
            p *= rho / rho_prev
            p += z
        else:
            p = z.copy()
        q = matvec(p)
        alpha = rho / dot(p, q)
        x += alpha * p
        r -= alpha * q
        rho_prev = rho
        if callback:
            callback(x)
    return x, maxiter


def run_oracle(kind, N, **kw):
    """The same case on the CPU oracle (GN: with exactly rounded CG dot products)."""
    from oracle import gnk_oracle as O
    prob, y, u0 = O.bratu_workload(N)
    norms, nfevs, cgs = [], [], []

    def cb(x, nfev, cg_iter):
        norms.append(float(np.linalg.norm(x)))
        nfevs.append(nfev)
        cgs.append(cg_iter)

    res, jac = prob.make_res(y), prob.make_jac()
    orig = O.scipy_cg
    with contextlib.redirect_stdout(io.StringIO()) as out:
        if kind == "gnk":
            r = O.gauss_newton_krylow(res, u0, jac, callback=cb, **kw)
        else:
            O.scipy_cg = exact_cg
            try:
                r = O.gauss_newton(res, u0, jac, callback=cb, **kw)
            finally:
                O.scipy_cg = orig
    return {"nit": r.nit, "nrev": r.nrev, "njev": r.njev, "success": bool(r.success), "nfev": nfevs,
            "cg_iter": cgs, "norms": norms, "stdout": out.getvalue()}


DEFAULT_ITERS = 45
ORACLE_FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "multislab_oracle.json")


def case_key(kind, kw):
    return kind + ":" + json.dumps(kw, sort_keys=True)


def cases_for(N, iters):
    """The solver cases run at grid N (GN unpreconditioned only where its sensitivity evidence exists)."""
    from tests import tolerances as T
    cases = [("gnk", dict(krylow_restart=20, max_iter=iters, version=v))
             for v in ("res_old", "res_new", "jac_old_res_old", "jac_old_res_new")]
    if f"gn{N}" in T.sensitivity():               # unpreconditioned GN: evidence recorded at grid 256
        cases.append(("gn", dict(max_iter=4, cg_rtol=1e-4)))
    cases.append(("gn", dict(max_iter=3, cg_rtol=1e-4, cg_preconditioner=True)))
    return cases


def oracle_result(kind, N, kw):
    """The oracle's run of a case: from the committed fixture (tests/golden/make_multislab_oracle.py,
    the same run_oracle) when it holds the case, else computed here."""
    if os.path.exists(ORACLE_FIXTURE):
        with open(ORACLE_FIXTURE) as f:
            got = json.load(f)["grids"].get(str(N), {}).get(case_key(kind, kw))
        if got is not None:
            return got
    return run_oracle(kind, N, **kw)


BACKEND = None          # --numpy: the NumPy test double of the C-ABI (CPU rehearsal of this script)


def _be():
    return None if BACKEND is None else BACKEND()


def run(kind, prob, y, u0, comm, **kw):
    norms, nfevs, cgs = [], [], []

    def cb(x, nfev, cg_iter):
        norms.append(float(np.linalg.norm(x)))
        nfevs.append(nfev)
        cgs.append(cg_iter)

    res, jac = prob.make_res(y), prob.make_jac()
    with contextlib.redirect_stdout(io.StringIO()) as out:
        if kind == "gnk":
            r = gnk.gauss_newton_krylow(res, u0, jac, callback=cb, comm=comm, _backend=_be(), **kw)
        else:
            r = gnk.gauss_newton(res, u0, jac, callback=cb, comm=comm, _backend=_be(), **kw)
    return {"nit": r.nit, "nrev": r.nrev, "njev": r.njev, "success": bool(r.success), "nfev": nfevs,
            "cg_iter": cgs, "norms": norms, "xnorm": float(np.linalg.norm(r.x)), "stdout": out.getvalue()}


def rel_diff(a, b):
    if len(a) != len(b) or not b:
        return float("inf")
    return float(np.max(np.abs(np.array(a) - np.array(b)) / np.abs(b)))


def staged_vs_host(prob, y_full, u0_full, comm, steps):
    """GNKSolver on per-rank staged inputs vs on full-grid host inputs: identical bits."""
    outs = []
    for staged in (True, False):
        dev = BratuDevice(prob, comm, backend=_be())
        if staged:
            u0, y, _ = slab_inputs(dev)
        else:
            u0, y = u0_full, y_full
        s = gnk.GNKSolver(prob, y, krylow_restart=20, max_iter=10 ** 6, comm=comm, backend=dev.backend)
        s.setup(u0)
        with contextlib.redirect_stdout(io.StringIO()):
            for _ in range(steps):
                if s.step():
                    break
        with contextlib.redirect_stdout(io.StringIO()):
            r = s.finish(result_format="torch")
        outs.append((r.x.cpu().numpy().copy() if torch.is_tensor(r.x) else np.asarray(r.x).copy(), s.nfev, [t["k"] for t in s.trace]))
    same = bool(np.array_equal(outs[0][0], outs[1][0]) and outs[0][1:] == outs[1][1:])
    return {"staged_equals_host_inputs": same, "steps": steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--iters", type=int, default=DEFAULT_ITERS)
    ap.add_argument("--out", required=True)
    ap.add_argument("--numpy", action="store_true")
    ap.add_argument("--transport", choices=("gloo", "shim"), default="gloo")
    ap.add_argument("--oracle", type=int, default=1)
    a = ap.parse_args()
    if a.numpy:
        global BACKEND
        from tests.numpy_backend import NumpyBackend
        BACKEND = NumpyBackend
    else:
        torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    N = a.grid
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    np.random.seed(42)
    u0 = prob.u_true + 0.1 * np.random.normal(loc=0, scale=1, size=N * N)
    one = BratuDevice(prob, Comm(single=True), backend=_be())          # y = F(u_true) on one rank
    F = one.vec()
    one.backend.forward(one.load(prob.u_true), F)
    y = F[one.slab.own].cpu().numpy().copy()
    del one, F
    cases = cases_for(N, a.iters)
    if a.transport == "shim":
        from tests.transport_shim import StagedTransportComm
        make_comm = StagedTransportComm
    else:
        make_comm = Comm
    comm = make_comm()
    mine = []
    for kind, kw in cases:
        print(f"[rank {rank}] {kind} {kw}", file=sys.stderr, flush=True)
        mine.append(run(kind, prob, y, u0, comm, **kw))
    staging = staged_vs_host(prob, y, u0, make_comm(), steps=24)
    shim_calls = getattr(comm, "staged_calls", None)
    every = [None] * world
    dist.all_gather_object(every, {"cases": mine, "staging": staging})
    dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        return 0
    report, ok = [], True
    keys = ("nit", "nrev", "njev", "success", "nfev", "cg_iter", "stdout")
    segmented = reduction_segments(N, world, None) > 0 and BACKEND is None   # the NumPy double has none
    for i, ((kind, kw), d) in enumerate(zip(cases, mine)):
        print(f"[rank 0] single-rank and oracle runs of case {i}: {kind} {kw}", file=sys.stderr, flush=True)
        ranks_equal = all(e["cases"][i] == d for e in every)
        s = run(kind, prob, y, u0, Comm(single=True, segments=segmented), **kw)
        same = all(d[f] == s[f] for f in keys)
        rel = rel_diff(d["norms"], s["norms"])
        tol = bound(kind, kw, N)
        bits = d["norms"] == s["norms"] and d["xnorm"] == s["xnorm"]
        case_ok = same and ranks_equal and (bits if segmented else rel <= tol)
        entry = {"case": kind, **kw, "world": world, "grid": N, "transport": a.transport, "segmented": segmented,
                 "ranks_identical": ranks_equal, "bookkeeping_equal": same, "bit_identical": bits,
                 "max_rel_norm_diff": rel, "tol": 0.0 if segmented else tol, "nit": s["nit"], "nrev": s["nrev"]}
        if a.oracle:
            o = oracle_result(kind, N, kw)
            o_keys = keys if kind == "gn" else ("nit", "nrev", "njev", "success", "nfev", "stdout")
            o_same = all(d[f] == o[f] for f in o_keys)
            o_rel = rel_diff(d["norms"], o["norms"])
            o_tol = oracle_bound(kind, kw, N)
            entry.update(oracle_bookkeeping_equal=o_same, oracle_max_rel_norm_diff=o_rel, oracle_tol=o_tol)
            case_ok = case_ok and o_same and o_rel <= o_tol
        entry["ok"] = case_ok
        ok &= case_ok
        report.append(entry)
    stage_ok = all(e["staging"]["staged_equals_host_inputs"] for e in every)
    ok &= stage_ok
    with open(a.out, "w") as f:
        json.dump({"ok": bool(ok), "world": world, "grid": N, "transport": a.transport, "staging_ok": stage_ok,
                   "shim_calls": shim_calls, "cases": report}, f, indent=1)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
