#!/bin/bash
# Round 3, session 2, GPU session H: the first-trial kernel on one workgroup per row segment (vjpgrow)
# vs the product's resident persistent grid; kbench trialp 8192^2, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2h
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
kb() {   # kb LIBTAG K
  local lib=$PWD/gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so
  [ "$1" != new ] && lib=$PWD/tools/_var/libgnk_$1.so
  GNK_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --k $2 --reps 9 --kernels trialp,vjpg | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/$/}/"
}
for rep in 1 2; do
  for k in 5 9 12 16 20; do
    for v in new vjpgrow; do
      step "trial_${v}_${k}_$rep" kb $v $k >> $O/trial_row_ab.jsonl
    done
  done
done
echo done
