#!/bin/bash
# Round 3 validation, part 1: smoke, then the -m gpu files other than the multi-rank / C4-C5 ones.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3t
mkdir -p $O
export TMPDIR=/tmp GNK_TEST_LOG_DIR=$PWD/$O/workers
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
echo "smoke ok $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solvers.py tests/test_gpu_generic.py tests/test_gpu_baseline_sizes.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$? $(date +%T)"
