"""Run a multi-rank test worker in fresh child processes (torch.distributed.run).  With
GNK_TEST_LOG_DIR set -- or on a gpurun box ($GRAFT_REPO_ROOT set), where it defaults to
gpurun_out/test_workers -- the workers' stderr (their progress lines) streams into a file there while
they run, so the box's watchdog sees progress during a long multi-rank case, and its tail is returned
on failure."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_workers(nproc, script, args, name, timeout):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nproc-per-node", str(nproc), os.path.join(ROOT, "tests", script), *map(str, args)]
    logdir = os.environ.get("GNK_TEST_LOG_DIR")
    if not logdir and os.environ.get("GRAFT_REPO_ROOT"):
        logdir = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out", "test_workers")
    if not logdir:
        p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
        return p.returncode, p.stderr[-4000:]
    os.makedirs(logdir, exist_ok=True)
    path = os.path.join(logdir, f"{name}.err")
    with open(path, "w") as err:
        p = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=err, timeout=timeout)
    with open(path) as f:
        return p.returncode, f.read()[-4000:]
