#!/bin/bash
# Round 3, GPU session R: k_gram_x for 2..4 column blocks (k = 21..63) vs the chunked / prefetching
# kernels (gnk_set_tuning(GNK_TUNE_GRAM_WIDE, 3)); kernel parity first; PMC of k = 33 / 51.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3r
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
for k in 21 27 33 40 47 51 57 63; do
  for w in 0 3; do
    step "wide_${w}_$k" timeout -k 10 150 python -u tools/kbench.py --k $k --reps 5 --kernels gram2 --tune gram_wide=$w > $O/w_${w}_$k.json
  done
done
for k in 33 51; do
  echo "== pmc k=$k $(date +%T)"
  bash tools/pmc.sh $O/k$k --k $k --reps 3 --kernels gram2 || { echo "pmc k=$k failed rc=$?"; exit 1; }
done
echo done
