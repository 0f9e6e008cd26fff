#!/bin/bash
# Round 3, session 2, GPU session C: the driver's round-end GPU steps as it runs them (smoke, then
# pytest -m gpu -x -q) with per-test durations: the multislab oracle side now comes from the committed
# fixture, the C4 worker adds GN + CGLS at 32768^2 on 8 ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
echo "smoke ok $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=30 --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(date +%T)"
tail -45 $O/pytest_gpu.log
exit $rc
