#!/bin/bash
# One GPU-box session: build, probes, GPU tests, smoke, bench, rocprof summary.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
run() { echo "== $1 ($(date +%T))"; }
if [[ $STEP == all || $STEP == test ]]; then
  run build && timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
  run probe && timeout -k 10 120 python tools/probe.py > gpurun_out/probe.json 2> gpurun_out/probe.err &&
  run smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
  run pytest && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
fi
if [[ $STEP == all || $STEP == dist ]]; then
  # several ranks on this one GPU (gloo, host-staged collectives) vs the single-rank solve
  run dist && timeout -k 10 600 torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 2 tests/multislab_worker.py --grid 256 --out gpurun_out/dist2.json > gpurun_out/dist2.log 2>&1 &&
  timeout -k 10 600 torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 3 tests/multislab_worker.py --grid 384 --out gpurun_out/dist3.json > gpurun_out/dist3.log 2>&1 || exit $?
fi
if [[ $STEP == all || $STEP == bench ]]; then
  run bench && timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
fi
if [[ $STEP == all || $STEP == prof ]]; then
  run rocprof && (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err") || exit $?
fi
echo "== done"
