#!/bin/bash
# Round 3, session 2, GPU session A: smoke, the whole -m gpu suite at HEAD (fresh build in this
# container), the driver's bench command.  Each step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
echo "smoke ok $(date +%T)"
timeout -k 10 840 python -u -m pytest tests -m gpu -q -s --durations=15 --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(date +%T)"
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "done $(date +%T)"
