"""``python bench.py --gpus N`` on the GPU box: the bench starts N ranks itself.

* gloo rehearsal (GNK_BENCH_BACKEND=gloo: the 2 ranks share the one MI355X, collectives staged through
  the host): the result line says n_gpus 2, transport gloo, a 2-rank slab partition, and the whole job's
  steps were timed.
* RCCL with more ranks than GPUs: refused with a non-zero exit, never measured as one rank.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env):
    e = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GNK_BENCH_BACKEND"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *args], env=e, cwd=ROOT,
                          capture_output=True, text=True, timeout=400)


def test_bench_gpus2_gloo_runs_two_ranks():
    p = _bench(["--gpus", "2", "--grid", "512", "--steps", "4", "--warmup", "2", "--repeats", "1",
                "--cpu-seconds", "0", "--cg-iters", "0", "--jvp-reps", "3"], GNK_BENCH_BACKEND="gloo")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]                   # rank 0 only
    r = json.loads(lines[0])
    print(json.dumps({k: r[k] for k in ("n_gpus", "value", "ms_per_step", "config")}))
    assert r["n_gpus"] == 2 and r["config"]["transport"] == "gloo" and r["config"]["parallelism"] == "slab2"
    assert r["steps"] == 4 and r["value"] > 0


def test_bench_gpus_beyond_node_under_rccl_fails_loudly():
    n = torch.cuda.device_count() + 1
    p = _bench(["--gpus", str(n), "--grid", "512", "--steps", "2", "--cpu-seconds", "0", "--cg-iters", "0"])
    assert p.returncode != 0, p.stdout[-2000:]
    assert "refusing to measure fewer ranks" in p.stderr, p.stderr[-2000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
