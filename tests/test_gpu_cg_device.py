"""The fused CGLS iteration with its scalar recurrence on the device (gnk_cg_scalars) on the
MI355X: bit for bit the host-scalar iteration (iterates and counts), with the lagged stopping read and with a
read every iteration, to convergence and at an iteration cap; and one host wait per iteration (was two).
Multi-rank (merged pairs, rank order): tests/test_gpu_multislab.py's GN cases and the C4 worker run this path."""
import numpy as np
import pytest

from tests.test_host_logic import _cg_paths

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,maxiter,pre", [(512, None, True), (512, 40, True), (256, None, False), (256, 0, False)])
def test_cg_device_scalars_bit_identical_hip(N, maxiter, pre):
    from gauss_newton_via_generalized_krylov_subspaces_amd._native import HipBackend
    import torch
    got = _cg_paths(lambda: HipBackend(torch.device("cuda", 0)), N=N, maxiter=maxiter, pre=pre)
    xh, ih = got["host"]
    print({k: v[1] for k, v in got.items()})
    for name in ("device_lagged", "device"):
        x, it = got[name]
        assert it == ih and np.array_equal(x, xh), (name, it, ih, np.abs(x - xh).max())


def test_cg_device_scalars_one_host_wait_per_iteration():
    from gauss_newton_via_generalized_krylov_subspaces_amd import BratuPdeProblem
    from gauss_newton_via_generalized_krylov_subspaces_amd.gauss_newton import BratuGNOps, DeviceCG
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
    from oracle import gnk_oracle as O
    _, y, u0 = O.bratu_workload(512)
    comm = Comm(single=True)
    ops = BratuGNOps(BratuPdeProblem(513, 5, 10), y, comm)
    u = ops.load(u0)
    r0 = ops.vec()
    ops.residual(u, r0)
    cg = DeviceCG(ops)
    w0 = comm.counters["host_wait"]
    _, it = cg.solve(u, r0, cg_rtol=1e-8, preconditioner=True, maxiter=60)
    waits = comm.counters["host_wait"] - w0
    print(f"{it} CG iterations, {waits} host waits")
    assert it == 60 and waits <= it + 3          # + ||b||, the initial r.r, the Jacobi set-up
