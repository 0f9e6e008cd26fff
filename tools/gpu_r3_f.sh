#!/bin/bash
# Round 3, GPU session F: staged Gram ring depth sweep (4 / 5 slots at two blocks per CU vs 6 / 8 slots
# at one block per CU): is the pass DMA-latency bound?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3f
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
for k in 10 12 14 16 17 20; do
  for R in 0 4 5 6 8; do
    step "ring_${R}_$k" timeout -k 10 120 python -u tools/kbench.py --k $k --reps 7 --kernels gram2 --tune gram_ring=$R | sed "s/^/{\"ring\": $R, \"r\": /; s/$/}/" >> $O/ring.jsonl
  done
done
echo done
