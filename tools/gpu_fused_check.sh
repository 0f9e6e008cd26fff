#!/bin/bash
# fused pass: kernel parity vs the NumPy double, then the A/B against the separate passes (k <= 13)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/fused_ab.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_kern.log 2>&1 || { echo KERNEL_TEST_FAIL; exit 1; }
FUSED_KS="${FUSED_KS:-9 11 12 13}" bash tools/fused_ab.sh || { echo AB_FAIL; exit 1; }
echo ok
