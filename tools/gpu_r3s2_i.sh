#!/bin/bash
# Round 3, session 2, GPU session I: the operator kernel tests with the two-row sizes (N = 512, 1024).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "operators or bitwise or adjoint" > $O/kernels.log 2>&1; rc=$?
tail -25 $O/kernels.log
exit $rc
