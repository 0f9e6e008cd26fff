#!/bin/bash
# Round 3, GPU session N: PMC passes (tools/pmc.sh) over the wide Gram kernels at 8192^2:
# k_gram_w (k = 33), k_gram_wp (k = 51), k_gram_x (k = 64, 80, 100).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3n
mkdir -p $O
for k in 33 51 64 80 100; do
  echo "== pmc k=$k $(date +%T)"
  bash tools/pmc.sh $O/k$k --k $k --reps 3 --kernels gram2 || { echo "pmc k=$k failed rc=$?"; exit 1; }
done
echo done
