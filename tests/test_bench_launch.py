"""bench.py's multi-rank launch: ``python bench.py --gpus N`` must run N ranks or refuse.

CPU tests: ``launch_ranks`` gives every child the torch.distributed.run environment and propagates a
failing rank's exit code (killing the others); bench.py refuses a WORLD_SIZE / --gpus mismatch and, under
RCCL, a node with fewer GPUs than --gpus (this container has none).  The real N-rank runs on the GPU are in
tests/test_gpu_bench_launch.py.
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CHILD_ENV = """
import json, os, sys
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
        "HSA_ENABLE_IPC_MODE_LEGACY")
with open(os.path.join(sys.argv[1], "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys}, f)
"""

CHILD_FAIL = """
import os, sys, time
if os.environ["RANK"] == "1":
    sys.exit(3)
time.sleep(120)
"""


def test_launch_ranks_environment(tmp_path):
    rc = bench.launch_ranks(3, [sys.executable, "-c", CHILD_ENV, str(tmp_path)])
    assert rc == 0
    got = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"] == [g["LOCAL_RANK"] for g in got]
    assert {g["WORLD_SIZE"] for g in got} == {"3"} == {g["LOCAL_WORLD_SIZE"] for g in got}
    assert {g["MASTER_ADDR"] for g in got} == {"127.0.0.1"}
    assert len({g["MASTER_PORT"] for g in got}) == 1 and int(got[0]["MASTER_PORT"]) > 0
    assert {g["HSA_ENABLE_IPC_MODE_LEGACY"] for g in got} == {"0"}


def test_launch_ranks_failure_propagates_and_kills_the_rest():
    t0 = time.time()
    rc = bench.launch_ranks(2, [sys.executable, "-c", CHILD_FAIL], grace_s=5.0)
    assert rc == 3
    assert time.time() - t0 < 60           # rank 0 (sleeping 120 s) was terminated, not waited for


def _bench(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GNK_BENCH_BACKEND"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=e, capture_output=True,
                          text=True, timeout=300)


def test_bench_refuses_world_mismatch():
    p = _bench(["--gpus", "2"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in p.stderr, p.stderr[-2000:]


def test_bench_refuses_too_few_gpus_under_rccl():
    """This container has no GPU: --gpus 2 under RCCL is refused before any rank starts."""
    import torch
    if torch.cuda.device_count() >= 2:
        import pytest
        pytest.skip("node has >= 2 GPUs")
    p = _bench(["--gpus", "2"])
    assert p.returncode != 0 and "refusing to measure fewer ranks" in p.stderr, p.stderr[-2000:]


def test_launcher_forwards_sigterm_to_every_rank(tmp_path):
    """A SIGTERM to ``python bench.py --gpus N`` (the driver's timeout) must end every rank, not orphan them
    in their own sessions."""
    import signal
    script = ("import sys, time; sys.path.insert(0, %r); import bench; "
              "sys.exit(bench.launch_ranks(2, [sys.executable, '-c', 'import time; time.sleep(120)']))" % ROOT)
    p = subprocess.Popen([sys.executable, "-c", script])
    time.sleep(3)
    p.send_signal(signal.SIGTERM)
    rc = p.wait(timeout=60)
    assert rc != 0
    out = subprocess.run(["ps", "-eo", "pid,args"], capture_output=True, text=True).stdout
    assert "time.sleep(120)" not in out
