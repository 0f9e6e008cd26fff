#!/bin/bash
# Round 3 validation, part 2: C2 (with the recorded tie range for its converged last step), C4, C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3u
mkdir -p $O
export TMPDIR=/tmp GNK_TEST_LOG_DIR=$PWD/$O/workers
timeout -k 10 300 python -u -m pytest tests/test_gpu_baseline_sizes.py -k c2_full -v -s --timeout 250 --timeout-method thread > $O/c2.log 2>&1
echo "c2 rc=$? $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_large_configs.py -v -s --timeout 900 --timeout-method thread > $O/large.log 2>&1
echo "large rc=$? $(date +%T)"
