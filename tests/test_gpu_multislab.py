"""Multi-slab HIP path on the GPU: 2, 3 and 8 ranks sharing the one MI355X, compared
with one rank and with the CPU oracle.

Each case starts fresh child processes (torch.distributed.run, gloo with host-staged collectives:
RCCL refuses two ranks on one device) that run the HIP kernels on real slabs -- row0 > 0,
halo-filled ghost rows, rank-ordered reductions -- for GNK (all four versions, restart 20) and GN
(with Jacobi; without it too at grid 256, where its sensitivity case is recorded), then compare with the single-rank solve (tests/multislab_worker.py):
bookkeeping and printed messages identical, every rank identical, per-iteration ||x_k|| within the
bounds the oracle sensitivity tests back; per-rank staged inputs (inputs.py) reproduce the full-grid
inputs' run bit for bit.  World 8 is the C4 rank count (8 x 32 rows of a 256^2 grid).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,grid,transport", [(2, 256, "gloo"), (2, 256, "shim"), (3, 384, "shim"),
                                                   (8, 256, "shim")])
def test_multislab_hip_matches_single_rank_and_oracle(world, grid, transport, tmp_path):
    """transport "gloo": host-staged collectives (Comm.stage); "shim": Comm's RCCL branches (device
    all-gathers, pinned read_async, gnk_rank_sum, device halos) over a host-staged transport."""
    out = tmp_path / "multislab.json"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nproc-per-node", str(world), os.path.join(ROOT, "tests", "multislab_worker.py"),
           "--grid", str(grid), "--out", str(out), "--transport", transport]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    rep = json.loads(out.read_text())
    print(json.dumps(rep))
    assert rep["world"] == world and rep["staging_ok"] and rep["transport"] == transport, rep
    if transport == "shim":
        assert rep["shim_calls"]["all_gather"] > 0 and rep["shim_calls"]["p2p"] > 0
    for c in rep["cases"]:
        assert c["ranks_identical"] and c["bookkeeping_equal"], c
        assert c["max_rel_norm_diff"] <= c["tol"], c
        assert c["oracle_bookkeeping_equal"] and c["oracle_max_rel_norm_diff"] <= c["oracle_tol"], c
    assert rep["ok"]
