#!/bin/bash
# Round 3, GPU session E: the trial kernel rework (exact widths, resident grid, LDS coefficients) vs
# the HEAD build; k_gram_s ablations (what the per-step barrier, the exp, the Gram step and the VALU
# tail cost); kernel parity tests; the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3e
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
kb() {   # kb LIBTAG K KERNELS
  local lib=$PWD/gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so
  [ "$1" != new ] && lib=$PWD/tools/_diag/libgnk_$1.so
  GNK_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --k $2 --reps 7 --kernels $3 | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/$/}/"
}
step kernels timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > $O/kernels.log 2>&1
for k in 9 12 13 16 17 20; do
  step "trial_head_$k" kb head $k trialp >> $O/trial_ab.jsonl
  step "trial_new_$k" kb new $k trialp >> $O/trial_ab.jsonl
done
for k in 10 12 16 17 20; do
  for v in new nobar noexp nogram notail; do
    step "gram_${v}_$k" kb $v $k gram2 >> $O/gram_abl.jsonl
  done
done
step bench timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo done
