#!/bin/bash
# Round 3, GPU session A: the changed kernel-choice tests (gnk_set_tuning), GN/CGLS with compensated
# pairs, C5 (16384^2, k -> 71) and C4 (32768^2, 8 ranks) at their sizes, then the fused-pass fault
# diagnostic (last: it may fault).  Every step has its own time limit; a timeout / abort / signal
# ends the session there.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3a
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
step kernels timeout -k 10 500 $PT --timeout 200 tests/test_gpu_kernels.py -k "gram_mfma or deterministic or cg_matvec" > $O/kernels.log 2>&1
step solvers timeout -k 10 500 $PT --timeout 300 tests/test_gpu_solvers.py tests/test_gpu_baseline_sizes.py -k "gn or c3 or cg" > $O/solvers.log 2>&1
step c5 timeout -k 10 600 $PT --timeout 550 tests/test_gpu_large_configs.py -k c5 > $O/c5.log 2>&1
step c4 timeout -k 10 960 $PT --timeout 940 tests/test_gpu_large_configs.py -k c4 > $O/c4.log 2>&1
step fused_diag timeout -k 10 150 env GNK_LIB=tools/_diag/libgnk_fused19.so python -u tools/fused_fault_diag.py 8192 15 10 > $O/fused_diag.log 2>&1
echo done
