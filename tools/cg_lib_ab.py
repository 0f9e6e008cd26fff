"""CG iteration time of the current libgnk.so (or GNK_LIB) at 8192^2: bench.py's gn_cg workload (CGLS of the first GN
step, Jacobi, rtol 1e-8, capped), fused scipy recurrence with device scalars; prints ms per CG iteration and the
final x's checksum (bits must match between builds that claim the same arithmetic).
    python tools/cg_lib_ab.py TAG [--iters 200] [--reps 3]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton import BratuGNOps, DeviceCG  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--grid", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    prob = gnk.BratuPdeProblem(a.grid + 1, 5, 10)
    comm = Comm(single=True)
    dev = BratuDevice(prob, comm)
    u0, y, _ = slab_inputs(dev)
    ops = BratuGNOps(prob, y, comm, backend=dev.backend)
    u = ops.load(u0)
    r0 = ops.vec()
    ops.residual(u, r0)
    cg = DeviceCG(ops)
    cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=5)
    for rep in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x, it = cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=a.iters)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        xs = x[dev.slab.own].cpu().numpy()
        print(json.dumps({"tag": a.tag, "rep": rep, "iters": it, "ms_per_iter": 1e3 * el / it,
                          "x_sum": float(np.sum(xs)), "x_bits": int(np.bitwise_xor.reduce(xs.view(np.int64)))}),
              flush=True)


if __name__ == "__main__":
    main()
