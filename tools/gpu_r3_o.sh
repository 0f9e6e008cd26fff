#!/bin/bash
# Round 3, GPU session O: the marching 8-wave k_gram_x (5..7 column blocks, RinvAug in VGPRs, one workgroup per
# CU) -- kernel parity, then A/B vs the pair-split k_gram at 8192^2, k = 64..100.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3o
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
step kernels timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gram" > $O/kernels.log 2>&1
grep -q " passed" $O/kernels.log && ! grep -q "failed" $O/kernels.log || { echo "kernel tests failed"; exit 1; }
for k in 64 80 100; do
  for w in 0 3; do
    step "wide_${w}_$k" timeout -k 10 150 python -u tools/kbench.py --k $k --reps 5 --kernels gram2 --tune gram_wide=$w > $O/w_${w}_$k.json
  done
done
echo done
echo done
