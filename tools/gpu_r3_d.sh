#!/bin/bash
# Round 3, GPU session D: fused pass at k <= 19 (the tests round 2 removed, and the kbench sequence that
# "faulted"), the 8192^2 full-cycle parity test, then where the step time goes: rocprofv3 kernel
# trace + stats of the driver's bench command, SQ counters of the staged Gram (k = 16, 20) and the
# first-trial kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3d
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  "$@"; local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  if [ $rc -ge 124 ]; then echo "FATAL at $name"; exit $rc; fi
  return 0
}
step fused timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py > $O/fused.log 2>&1
step fused_diag timeout -k 10 150 python -u tools/fused_fault_diag.py 8192 15 10 > $O/fused_diag.log 2>&1
step rocprof bash tools/rocprof_bench.sh
step sq16 bash tools/pmc_sq.sh gpurun_out/r3d/sq16 --k 16 --reps 5 --kernels gram2
step sq20 bash tools/pmc_sq.sh gpurun_out/r3d/sq20 --k 20 --reps 5 --kernels gram2
step sqtrial bash tools/pmc_sq.sh gpurun_out/r3d/sqtrial --k 16 --reps 5 --kernels trialp
echo done
