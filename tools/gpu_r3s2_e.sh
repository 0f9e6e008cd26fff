#!/bin/bash
# Round 3, session 2, GPU session E: k_jvp A/B (bench metric's JVP half) -- non-temporal stores of J v,
# a grid of the resident workgroups, both -- vs the product build, interleaved twice; 8192^2 and 16384^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2e
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
kb() {   # kb LIBTAG GRID
  local lib=$PWD/gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so
  [ "$1" != new ] && lib=$PWD/tools/_var/libgnk_$1.so
  GNK_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --grid $2 --k 4 --reps 30 --kernels jvp,resid | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/$/}/"
}
for rep in 1 2; do
  for g in 8192 16384; do
    for v in new jvpnt jvpres jvpntres; do
      step "jvp_${v}_${g}_$rep" kb $v $g >> $O/jvp_ab.jsonl
    done
  done
done
echo done
