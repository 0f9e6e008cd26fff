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
  * multi-rank vs single-rank: bookkeeping identical, per-iteration ||x_k|| within TOL[case], each
    bound backed by a committed oracle sensitivity test (tests/test_oracle_sensitivity.py);
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
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402

# ||x_k|| bound, multi-rank vs single-rank (every reduction summed in a different order): GNK at
# max(1e-10, the spread of the reference's own arithmetic reordered as 2 .. 8 slabs order it, permuted
# QR, exact k = 1 sums, 1 vs 8 BLAS threads -- tests/tolerances.py, cases multislab<grid>_<version>);
# GN + CGLS at max(1e-10, the spread of the reference's GN with its CG dot products summed in other
# orders -- pairwise, reversed, 2 .. 8 slab blocks, 8 BLAS threads: cases gn<grid>[_pre]).
def bound(kind, kw, grid):
    from tests import tolerances as T
    if kind == "gnk":
        return T.trajectory_bound(f"multislab{grid}_{kw['version']}")
    return T.trajectory_bound(f"gn{grid}" + ("_pre" if kw.get("cg_preconditioner") else ""))


BACKEND = None          # --numpy: the NumPy test double of the C-ABI (CPU rehearsal of this script)


def _be():
    return None if BACKEND is None else BACKEND()


def run(kind, prob, y, u0, comm, **kw):
    norms, nfevs = [], []

    def cb(x, nfev, cg_iter):
        norms.append(float(np.linalg.norm(x)))
        nfevs.append(nfev)

    res, jac = prob.make_res(y), prob.make_jac()
    with contextlib.redirect_stdout(io.StringIO()) as out:
        if kind == "gnk":
            r = gnk.gauss_newton_krylow(res, u0, jac, callback=cb, comm=comm, _backend=_be(), **kw)
        else:
            r = gnk.gauss_newton(res, u0, jac, callback=cb, comm=comm, _backend=_be(), **kw)
    return {"nit": r.nit, "nrev": r.nrev, "njev": r.njev, "success": bool(r.success), "nfev": nfevs,
            "norms": norms, "xnorm": float(np.linalg.norm(r.x)), "stdout": out.getvalue()}


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
    ap.add_argument("--iters", type=int, default=45)
    ap.add_argument("--out", required=True)
    ap.add_argument("--numpy", action="store_true")
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
    cases = [("gnk", dict(krylow_restart=20, max_iter=a.iters, version=v))
             for v in ("res_old", "res_new", "jac_old_res_old", "jac_old_res_new")]
    from tests import tolerances as T
    if f"gn{N}" in T.sensitivity():               # unpreconditioned GN: evidence recorded at grid 256
        cases.append(("gn", dict(max_iter=4, cg_rtol=1e-4)))
    cases.append(("gn", dict(max_iter=3, cg_rtol=1e-4, cg_preconditioner=True)))
    mine = [run(kind, prob, y, u0, Comm(), **kw) for kind, kw in cases]
    staging = staged_vs_host(prob, y, u0, Comm(), steps=24)
    every = [None] * world
    dist.all_gather_object(every, {"cases": mine, "staging": staging})
    dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        return 0
    report, ok = [], True
    for i, ((kind, kw), d) in enumerate(zip(cases, mine)):
        ranks_equal = all(e["cases"][i] == d for e in every)
        s = run(kind, prob, y, u0, Comm(single=True), **kw)
        same = all(d[f] == s[f] for f in ("nit", "nrev", "njev", "success", "nfev", "stdout"))
        rel = float(np.max(np.abs(np.array(d["norms"]) - np.array(s["norms"])) / np.abs(s["norms"]))) \
            if len(d["norms"]) == len(s["norms"]) and s["norms"] else float("inf")
        tol = bound(kind, kw, N)
        case_ok = same and ranks_equal and rel <= tol
        ok &= case_ok
        report.append({"case": kind, **kw, "world": world, "grid": N, "ranks_identical": ranks_equal,
                       "bookkeeping_equal": same, "max_rel_norm_diff": rel, "tol": tol, "ok": case_ok,
                       "nit": s["nit"], "nrev": s["nrev"]})
    stage_ok = all(e["staging"]["staged_equals_host_inputs"] for e in every)
    ok &= stage_ok
    with open(a.out, "w") as f:
        json.dump({"ok": bool(ok), "world": world, "grid": N, "staging_ok": stage_ok, "cases": report}, f, indent=1)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
