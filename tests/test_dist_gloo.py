"""Multi-rank slab path on CPU: torch.distributed gloo, world sizes 2 and 3.

Each rank owns a slab of grid rows; the solver's halo exchanges and rank-ordered
reductions must reproduce the single-rank run (bookkeeping exactly, iterates to
1e-10) -- the same property the 8-GPU RCCL run relies on.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, method, kw, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _body(rank, world, method, kw, q)
    except BaseException as e:  # report instead of leaving the peer hanging
        q.put((rank, "error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _body(rank, world, method, kw, q):
    if True:
        import contextlib
        import io

        import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
        from tests.numpy_backend import NumpyBackend
        arr = dict(np.load(os.path.join(ROOT, "tests", "golden", "golden.npz")))
        prob = gnk.BratuPdeProblem(25, 5, 10)
        fn = gnk.gauss_newton_krylow if method == "gnk" else gnk.gauss_newton
        norms = []

        def cb(x, nfev, cg_iter):
            norms.append((float(np.linalg.norm(x)), nfev, cg_iter))

        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            out = fn(prob.make_res(arr["bratu24_y"]), arr["bratu24_u0"], prob.make_jac(), callback=cb,
                     _backend=NumpyBackend(), **kw)
        q.put((rank, out.nit, out.nrev, out.njev, out.success, out.x, norms, buf.getvalue()))


def _run(world, method, kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, method, kw, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = []
    for _ in procs:
        o = q.get(timeout=300)
        if o[1] == "error":
            for p in procs:
                p.kill()
            raise AssertionError(f"rank {o[0]} failed: {o[2]}")
        outs.append(o)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(outs, key=lambda o: o[0])


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("method,kw", [("gnk", {"version": "res_old", "max_iter": 30}),
                                       ("gnk", {"version": "res_new", "max_iter": 45, "krylow_restart": 20}),
                                       ("gn", {}), ("gn", {"cg_variant": "single_reduction"})])
def test_multi_rank_matches_golden(golden, world, method, kw):
    meta, arr = golden
    outs = _run(world, method, kw)
    # every rank took identical control decisions
    for o in outs[1:]:
        assert o[1:5] == outs[0][1:5]
        assert [n[1:] for n in o[6]] == [n[1:] for n in outs[0][6]]
        np.testing.assert_array_equal(o[5], outs[0][5])
    name = {"gnk": "bratu24_{version}_r{restart}", "gn": "bratu24_gn"}[method].format(
        version=kw.get("version"), restart=kw.get("krylow_restart"))
    case = meta["cases"][name]
    ref = case["per_iter"]
    n = len(outs[0][6])
    assert [x[1] for x in outs[0][6]] == ref["nfev"][:n]
    assert [x[2] for x in outs[0][6]] == ref["cg_iter"][:n]
    np.testing.assert_allclose([x[0] for x in outs[0][6]], ref["xnorm"][:n], rtol=1e-10)
    if method == "gn" or kw.get("max_iter", 100) == 100:
        assert outs[0][1:5] == (case["nit"], case["nrev"], case["njev"], case["success"])


def _staging_worker(rank, world, port, q):
    """inputs.slab_inputs on each rank (no full-grid vector anywhere) vs slices of the full-grid
    workload; Comm.gather_rows (tensor all-gather) reassembles the full vector."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
        from gauss_newton_via_generalized_krylov_subspaces_amd import inputs
        from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
        from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
        from tests.numpy_backend import NumpyBackend
        inputs.CHUNK = 1000                  # several chunks per slab at this size
        N = 61
        prob = gnk.BratuPdeProblem(N + 1, 5, 10)
        dev = BratuDevice(prob, Comm(), backend=NumpyBackend())
        u0, y, ut = inputs.slab_inputs(dev)
        np.random.seed(42)
        u0_full = prob.u_true + 0.1 * np.random.normal(loc=0, scale=1, size=N * N)
        y_full = dev.slab.to_host(dev.load(y))                # gather_rows over the tensor all-gather
        u0_back = dev.slab.to_host(dev.load(u0))
        q.put((rank, np.array_equal(u0_back, u0_full),
               np.array_equal(u0.data.numpy(), dev.load(u0_full).numpy()),
               np.array_equal(ut.data.numpy(), dev.load(prob.u_true).numpy()),
               y_full, y.data.numpy(), dev.load(y_full).numpy()))
    except BaseException as e:
        q.put((rank, "error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_slab_input_staging(world):
    """C4 input staging: per-rank slabs of u_true / u0 (streamed RNG) / y = F(u_true)
    (forward on the slab + halo) equal the full-grid workload's slabs bit for bit, ghost rows included."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_staging_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=300) for _ in procs], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
    for o in outs:
        assert o[1] != "error", o
        assert o[1] and o[2] and o[3]
        np.testing.assert_array_equal(o[5], o[6])            # y's ghost rows == the full vector's rows
    import gauss_newton_via_generalized_krylov_subspaces_amd as gnk
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
    from tests.numpy_backend import NumpyBackend
    prob = gnk.BratuPdeProblem(62, 5, 10)
    one = BratuDevice(prob, Comm(single=True), backend=NumpyBackend())
    F = one.vec()
    one.backend.forward(one.load(prob.u_true), F)
    np.testing.assert_array_equal(outs[0][4], F[one.slab.own].numpy())   # the same F as one rank computes


def _sum_max_pairs_worker(rank, world, port, q):
    """Comm.sum_max_pairs (the restart step's single read) against sum_max on each pair: the same sums in
    tree_sum's order, the same NaN-propagating max."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
        comm = Comm()
        rng = np.random.default_rng(100 + rank)
        vals = [float(rng.standard_normal()) * 10.0 ** int(rng.integers(-8, 8)) for _ in range(4)]
        if rank == world - 1:
            vals[3] = float("nan")                # a NaN max on one rank wins
        t = torch.tensor(vals + [7.0, 7.0], dtype=torch.float64)
        both = comm.sum_max_pairs(t, 2)
        one = [comm.sum_max(torch.tensor(vals[0:2], dtype=torch.float64)),
               comm.sum_max(torch.tensor(vals[2:4], dtype=torch.float64))]
        q.put((rank, both, one))
    except BaseException as e:
        q.put((rank, "error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sum_max_pairs_equals_sum_max(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sum_max_pairs_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=300) for _ in procs], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
    for o in outs:
        assert o[1] != "error", o
        (s0, m0), (s1, m1) = o[1]
        (t0, n0), (t1, n1) = o[2]
        assert s0 == t0 and m0 == n0 and s1 == t1
        assert np.isnan(m1) and np.isnan(n1)
    assert all(o[1][0] == outs[0][1][0] for o in outs)     # every rank the same decision inputs
