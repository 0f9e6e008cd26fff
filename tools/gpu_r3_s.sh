#!/bin/bash
# Round 3, GPU session S: persistent residual / pending-GEMV grids, k = 8 on the one-point VALU Gram:
# kernel parity, the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s
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
step kernels timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/kernels.log 2>&1
grep -q " passed" $O/kernels.log && ! grep -q "failed" $O/kernels.log || { echo "kernel tests failed"; exit 1; }
step resid timeout -k 10 120 python -u tools/kbench.py --k 8 --reps 9 --kernels resid,gram2 > $O/kb.json
step bench timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo done
