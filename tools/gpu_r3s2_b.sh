#!/bin/bash
# Round 3, session 2, GPU session B: the -m gpu tests after test_gpu_large_configs (session A was cut
# off by the silence watchdog inside the multi-rank cases: worker logs now stream to gpurun_out), then
# the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_multislab.py tests/test_gpu_solvers.py -m gpu -v -s --durations=20 --timeout 600 --timeout-method thread > $O/pytest_gpu_rest.log 2>&1; rc=$?
echo "pytest rc=$rc $(date +%T)"
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "done $(date +%T)"
