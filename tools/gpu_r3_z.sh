#!/bin/bash
# Round 3, GPU session Z: the trial kernel marching contiguous row ranges (r rows carried in registers)
# vs the HEAD build (row-strided grid); kernel parity tests; the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3z
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
  [ "$1" != new ] && lib=$PWD/tools/_var/libgnk_$1.so
  GNK_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --k $2 --reps 7 --kernels $3 | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/$/}/"
}
step kernels timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemv or vjp" > $O/kernels.log 2>&1
for k in 5 9 12 16 17 20; do
  step "trial_head_$k" kb head $k trialp >> $O/trial_ab.jsonl
  step "trial_new_$k" kb new $k trialp >> $O/trial_ab.jsonl
done
step bench timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err

GNK_LIB=$PWD/tools/_var/libgnk_head.so step bench_head timeout -k 10 300 python -u bench.py --cpu-seconds 0 > $O/bench_head.json 2> $O/bench_head.err
step bench2 timeout -k 10 300 python -u bench.py --cpu-seconds 0 > $O/bench2.json 2> $O/bench2.err
echo done
