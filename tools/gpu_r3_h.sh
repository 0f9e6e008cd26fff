#!/bin/bash
# Round 3, GPU session H: staged Gram with the jdiag batched over 4 rows (R = 4) vs the 5-slot ring.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3h
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
for k in 10 12 14 16 17 20; do
  for R in 0 5; do
    step "gram_${R}_$k" timeout -k 10 120 python -u tools/kbench.py --k $k --reps 7 --kernels gram2 --tune gram_ring=$R > $O/g_${R}_$k.json
  done
done
step bench timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo done
