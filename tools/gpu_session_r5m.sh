#!/bin/bash
# Round-5: read-g chunk width of the wide vjp_gemv_t split (product 32 columns vs 16 / 24 builds), kbench vjpg
# at 16384^2, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for i in 1 2; do
  for k in 40 57 100; do
    timeout -k 10 300 python3 tools/kbench.py --grid 16384 --k $k --reps 5 --kernels vjpg | sed "s/^/b32 k=$k /" || exit 1
    for W in 16 24; do
      GNK_LIB=tools/_var/libgnk_b$W.so timeout -k 10 300 python3 tools/kbench.py --grid 16384 --k $k --reps 5 --kernels vjpg | sed "s/^/b$W k=$k /" || exit 1
    done
  done
done
