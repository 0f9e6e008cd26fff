#!/bin/bash
# Round 3, session 2, GPU session D: k_gram_v1 (k = 8, 9) A/B -- the transform in LDS capped at two waves
# per SIMD (v1lds), the next row's loads one row ahead (v1pf, one wave per SIMD) -- vs the product
# build; the generic-problem GPU tests (new graded-spectrum dense case).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2d
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
  GNK_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --k $2 --reps 9 --kernels gram2 | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/$/}/"
}
step generic timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_generic.py > $O/generic.log 2>&1
for k in 7 8 9; do
  for v in new v1lds v1pf; do
    step "gram_${v}_$k" kb $v $k >> $O/v1_ab.jsonl
  done
done
for k in 8 9; do step "gram_new2_$k" kb new $k >> $O/v1_ab.jsonl; step "gram_v1lds2_$k" kb v1lds $k >> $O/v1_ab.jsonl; done
echo done
