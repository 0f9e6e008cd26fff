#!/bin/bash
# Round 3, session 2, GPU session G: the two-row JVP / VJP / forward / residual kernels in the product --
# smoke, the whole -m gpu suite (-x, as the driver runs it), the driver's bench command, and the
# rocprofv3 kernel trace + stats of that command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
echo "smoke ok $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=10 --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(date +%T)"; tail -14 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "bench ok $(date +%T)"
bash tools/rocprof_bench.sh || exit $?
echo "done $(date +%T)"
