#!/bin/bash
# Round-end GPU session: smoke, the whole -m gpu suite (no -x: every failure listed), the driver's
# bench command, the capped C5 point.  Each step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1; echo "pytest rc=$?"
timeout -k 10 600 python bench.py --warmup 5 > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
if [[ ${C5:-1} == 1 ]]; then
  timeout -k 10 600 python bench.py --grid 16384 --restart 100 --steps 99 --warmup 1 --repeats 1 --cpu-seconds 0 --cg-iters 0 --jvp-reps 2 > gpurun_out/bench_c5_final.json 2> gpurun_out/bench_c5_final.err; echo "c5 rc=$?"
fi
echo done
