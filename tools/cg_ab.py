"""A/B of the fused CGLS iteration at 8192^2 (bench.py's gn_cg workload): host scalars (_cg_fused) vs device
scalars (gnk_cg_scalars) with and without the lagged read.  Prints ms per CG iteration per variant (JSON lines)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton import BratuGNOps, DeviceCG  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402


def main(N=8192, iters=100, reps=2):
    torch.cuda.set_device(0)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    comm = Comm(single=True)
    dev = BratuDevice(prob, comm)
    u0, y, _ = slab_inputs(dev)
    ops = BratuGNOps(prob, y, comm, backend=dev.backend)
    u = ops.load(u0)
    r0 = ops.vec()
    ops.residual(u, r0)
    cg = DeviceCG(ops)
    for rep in range(reps):
        for name, ds, lag in (("host", False, False), ("device_lagged", True, True), ("device", True, False)):
            cg.device_scalars, cg.lag_reads = ds, lag
            cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=5)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _, it = cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=iters)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(json.dumps({"variant": name, "rep": rep, "iters": it, "ms_per_iter": 1e3 * el / it}), flush=True)


if __name__ == "__main__":
    main()
