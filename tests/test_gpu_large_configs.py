"""BASELINE.json's two largest configurations at their sizes, on the one MI355X of a test box.

* C4 (configs[3]): Bratu 32768^2 row-partitioned over 8 ranks -- all eight on cuda:0, collectives
  through slab.Comm's RCCL code paths with a host-staged transport (tests/c4_worker.py,
  tests/transport_shim.py); krylow_restart 20, the first 6 outer iterations; 8 ranks vs 1 rank on the same
  inputs, both with reduction segments (gnk_set_segments): identical decisions, bookkeeping and
  per-iteration ||x_k||^2 / ||r_k||^2 bit for bit on every rank and vs one rank.  (The reference
  itself cannot run at this size; the oracle pins the algorithm at
  smaller sizes: tests/test_gpu_multislab.py, tests/test_gpu_baseline_sizes.py.)  The same worker then
  runs GN + Jacobi CGLS (rtol 1e-8, each CG run capped at 40 iterations, 2 outer iterations) at 32768^2
  on 8 ranks vs 1 rank -- SURVEY §8 f2's "C3 at 32768^2": cg_iter, nfev, step lengths, ||x_k|| and
  ||r_k|| bit for bit (compensated CG scalars merged across ranks before rounding; the rest segmented).
* C5 (configs[4]): Bratu 16384^2 with the basis growing without restart (krylow_restart 100,
  ref:gauss_newton_krylow.py:81-82, ref:krylow.py:72-73) to k = 99 -- through every Gram kernel of
  the wide path: the staged MFMA pass (k <= 31; k_gram_q on 4x4x4 blocks from k = 8) and the marching wide
  pass (k_gram_x, 32..99; V = 101 x 2.15 GB = 217 GB).
  k >= 112 (the pair-split k_gram, C5's range on 8 GPUs) is covered against the NumPy Gram at small N
  (tests/test_gpu_kernels.py::test_gram_mfma).  k = 200 does not fit one GPU
  (the basis alone is 429 GB); the full-size run is checked by properties:
    - the reference basis (sc_j V_j, krylow.py) is orthonormal: max |V^T V - I| <= ORTH_TOL, computed on
      the device (gnk_flat_gemv_t);
    - every least-squares solve accepted its factor with cond(R_Y) <= lls.COND_ACCEPT;
    - a second run from the same inputs reproduces every per-iteration norm and counter bit for bit.
"""
import contextlib
import io
import json

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.inputs import slab_inputs  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.lls import COND_ACCEPT  # noqa: E402
from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm  # noqa: E402
from tests._subproc import run_workers  # noqa: E402

# CGS1 (ref:krylow.py:64) loses orthogonality ~ u / rho_j on a column whose projection removed most of
# g (rho_j = ||w_j|| / ||g_j||); measured here at 16384^2 (see the printed value)
ORTH_TOL = 1e-12


def test_c4_32768_eight_ranks_on_one_gpu(tmp_path):
    out = tmp_path / "c4.json"
    rc, err = run_workers(8, "c4_worker.py", ["--out", out], "c4_32768_8ranks", timeout=900)
    assert rc == 0, err
    rep = json.loads(out.read_text())
    print(json.dumps({k: v for k, v in rep.items() if k not in ("multi", "single")}))
    print("multi:", json.dumps(rep["multi"]))
    assert rep["world"] == 8 and rep["grid"] == 32768
    assert rep["ranks_identical"] and rep["bookkeeping_equal"], rep
    print("per-iteration rel ||x_k|| diff", rep["rel_xnorm_diff"], "bit identical", rep["bit_identical"])
    assert rep["bit_identical"] and rep["max_rel_rnorm_diff"] == 0.0 and rep["max_rel_xnorm_diff"] == 0.0, rep
    assert rep["shim_calls"]["all_gather"] > 0 and rep["shim_calls"]["p2p"] > 0
    # GN + CGLS at the same size and partition (C3 at 32768^2), 8 ranks vs 1, bit for bit
    gn = rep["gn"]
    print("GN multi:", json.dumps({k: v for k, v in gn["multi"].items() if k != "stdout"}))
    print(f"GN: bit-identical {gn['bit_identical']}, ranks identical {gn['ranks_identical']}, "
          f"max rel ||r_k|| diff {gn['max_rel_rnorm_diff']:.3g}, {gn['seconds_multi']:.1f} s on 8 ranks")
    print("GN collectives / host waits per CG iteration on 8 ranks:", json.dumps(gn["comm_per_cg_iter_multi"]))
    assert gn["comm_per_cg_iter_multi"]["host_wait"] <= 1.5      # device CG scalars: one (lagged) read per iteration
    assert gn["ranks_identical"] and gn["bit_identical"], gn
    assert gn["max_rel_rnorm_diff"] == 0.0 and gn["ok"], gn
    assert rep["ok"]


def test_c5_k200_eight_ranks_on_one_gpu(tmp_path):
    """C5's basis growth to k = 200 on C5's 8 ranks (tests/c5_worker.py: 8192^2, no restart, V = 108 GB; C5's
    own 16384^2 basis is 429 GB, the 8 GPUs' HBM): every wide Gram kernel in turn, including the pair-split
    k_gram for k >= 112, with (k+1)^2 Grams all-gathered and rank-summed through slab.Comm's RCCL branches
    (host-staged transport), then one rank over the whole grid.  Asserted: identical decisions on every rank
    and vs one rank (ref:krylow.py:72-73 grows the basis every iteration, ref:gauss_newton_krylow.py:81-82
    never restarts), per-iteration ||x_k|| / ||r_k|| bit for bit while the basis is on the segmented kernels
    (iterations 1..31: iteration i solves on the k = i column basis, up to k = 31 with the segmented staged Gram
    pass; from k = 32 the Gram pass is a wide kernel that counts a segment fallback) and within 1e-12 after (the
    wide kernels reduce over their own slab
    decomposition), the one-rank reference basis orthonormal (max |V^T V - I| <= ORTH_TOL) and every accepted
    least-squares factor well conditioned (cond(R_Y) <= COND_ACCEPT, the threshold of a second CholeskyQR pass)."""
    out = tmp_path / "c5.json"
    rc, err = run_workers(8, "c5_worker.py", ["--out", out], "c5_8192_k200_8ranks", timeout=900)
    assert rc == 0, err
    rep = json.loads(out.read_text())
    print(json.dumps({k: v for k, v in rep.items() if k not in ("multi", "single", "rel_xnorm_diff", "rel_rnorm_diff")}))
    assert rep["world"] == 8 and rep["max_k"] == 200 and rep["single_basis_k"] == 201, rep["max_k"]
    assert rep["ranks_identical"] and rep["bookkeeping_equal"]
    ex, er = np.array(rep["rel_xnorm_diff"]), np.array(rep["rel_rnorm_diff"])
    assert ex.size == er.size == 200
    assert np.all(ex[:31] == 0.0) and np.all(er[:31] == 0.0), (ex[:31], er[:31])
    assert ex.max() <= 1e-12 and er.max() <= 1e-12, (ex.max(), er.max())
    assert rep["single_max_abs_VtV_minus_I"] <= ORTH_TOL
    assert rep["max_cond_multi"] <= COND_ACCEPT and rep["max_cond_single"] <= COND_ACCEPT


def _c5_run(N, max_iter):
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    comm = Comm(single=True)
    dev = BratuDevice(prob, comm)
    u0, y, _ = slab_inputs(dev)
    own = dev.slab.own
    rec = []

    def cb(x, nfev, cg_iter):
        rec.append((float(torch.linalg.norm(x.x[own])), float(x.sumsq), int(nfev)))

    s = gnk.GNKSolver(prob, y, krylow_restart=100, max_iter=max_iter, comm=comm, backend=dev.backend, callback=cb,
                      callback_format="device")
    with contextlib.redirect_stdout(io.StringIO()) as so:
        s.setup(u0)
        while not s.step():
            pass
        r = s.finish(result_format="torch")
    return s, dev, rec, (r.nit, r.nrev, r.njev, r.success, so.getvalue())


def test_c5_16384_wide_basis_properties():
    N, max_iter = 16384, 100       # steps 1..99 (k = 1..99; the restart would come after step 100)
    s, dev, rec, book = _c5_run(N, max_iter)
    b = s.basis
    k = b.k
    ks = [t["k"] for t in s.trace]
    print(f"C5 16384^2: nit {book[0]} nrev {book[1]} basis k = {k}, per-step k {ks[0]}..{ks[-1]}")
    assert book[0] == max_iter - 1 and k >= 99 and max(ks) >= 99          # k_gram_x ran up to k = 99
    # orthonormality of the reference basis, on the device (whole slab: the exterior ghost rows are 0)
    be = dev.backend
    h = be.zeros(k)
    G = np.zeros((k, k))
    for j in range(k):
        be.flat_gemv_t(b.V, k, b.V[j], h)
        G[:, j] = h.cpu().numpy()
    sc = b.sc[:k]
    G = sc[:, None] * G * sc[None, :]
    orth = float(np.max(np.abs(G - np.eye(k))))
    worst = np.unravel_index(np.argmax(np.abs(G - np.eye(k))), G.shape)
    print(f"C5: max |V^T V - I| = {orth:.3g} at {worst}; diagonal within {np.max(np.abs(np.diag(G) - 1)):.3g}")
    # cross-check of the device GEMV^T against rocBLAS (torch fp64 matmul) on the first columns
    Vs = b.V[:8] * torch.as_tensor(sc[:8], device=b.V.device)[:, None]
    G8 = (Vs @ Vs.T).cpu().numpy()
    print(f"C5: first 8 columns, |G_gemv_t - G_torch| max {np.max(np.abs(G8 - G[:8, :8])):.3g}")
    del Vs
    # every accepted least-squares factor was well conditioned
    conds = [h_[2][-1] for h_ in s.lls.history if h_[2]]
    extra = sum(1 for h_ in s.lls.history if h_[1] > 1)
    print(f"C5: {len(conds)} solves, max accepted cond(R_Y) {max(conds):.3g}, {extra} with more than one pass")
    nsolves = len(s.lls.history)
    del s, h, b, dev
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    # determinism: the whole run again, every per-iteration scalar bit for bit
    s2, _, rec2, book2 = _c5_run(N, max_iter)
    print(f"C5 rerun: bookkeeping equal {book2 == book}, per-iteration scalars equal {rec2 == rec}")
    assert book2 == book and rec2 == rec
    assert len(conds) == nsolves and max(conds) <= COND_ACCEPT
    assert orth <= ORTH_TOL
