#!/bin/bash
# Round 3, GPU session K: C4 (32768^2, 8 ranks on one MI355X through the RCCL-path shim) vs one rank.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3k
mkdir -p $O
export TMPDIR=/tmp GNK_TEST_LOG_DIR=$PWD/$O/workers
echo "== c4 $(date +%T)"
timeout -k 10 1050 python -u -m pytest -x -v -s --timeout 1000 --timeout-method thread tests/test_gpu_large_configs.py -k c4 > $O/c4.log 2>&1
echo "== c4 rc=$? $(date +%T)"
