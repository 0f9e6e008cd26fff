#!/bin/bash
# Round 3, GPU session B: staged-Gram halo fix (kernel tests + the kbench sequence that faulted),
# C5 and C4 at their sizes, the multi-slab tests (gloo and the RCCL-path shim, vs one rank and the
# oracle).  Each step has its own time limit; a timeout / abort / signal ends the session there.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3b
mkdir -p $O
export TMPDIR=/tmp GNK_TEST_LOG_DIR=$PWD/$O
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  "$@"; local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  if [ $rc -ge 124 ]; then echo "FATAL at $name"; exit $rc; fi
}
PT="python -u -m pytest -q -s --timeout-method thread"
step kernels timeout -k 10 300 $PT --timeout 200 tests/test_gpu_kernels.py tests/test_gpu_generic.py -k "gram or flat or generic" > $O/kernels.log 2>&1
step fused_diag timeout -k 10 150 python -u tools/fused_fault_diag.py 8192 15 10 > $O/fused_diag.log 2>&1
step c5 timeout -k 10 600 $PT --timeout 550 tests/test_gpu_large_configs.py -k c5 > $O/c5.log 2>&1
step c4 timeout -k 10 960 $PT --timeout 940 tests/test_gpu_large_configs.py -k c4 > $O/c4.log 2>&1
step multislab timeout -k 10 1100 $PT --timeout 620 tests/test_gpu_multislab.py > $O/multislab.log 2>&1
echo done
