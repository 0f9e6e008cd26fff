#!/bin/bash
# Round 3, GPU session C: the software-pipelined staged Gram kernel -- kernel parity tests, then the
# per-k A/B at 8192^2 against the previous build (tools/_diag/libgnk_base.so), then the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3c
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  "$@"; local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  if [ $rc -ge 124 ]; then echo "FATAL at $name"; exit $rc; fi
  return $rc
}
step kernels timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gram" > $O/kernels.log 2>&1 || exit 1
step fused timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py > $O/fused.log 2>&1
step fused_diag timeout -k 10 150 python -u tools/fused_fault_diag.py 8192 15 10 > $O/fused_diag.log 2>&1
step solvers timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_solvers.py tests/test_gpu_baseline_sizes.py -k "c2 or headline or bratu" > $O/solvers.log 2>&1
: > $O/gram_ab.jsonl
for k in ${KS:-4 8 9 10 12 13 14 16 17 18 20}; do
  step "ab_new_$k" timeout -k 10 120 python tools/kbench.py --k $k --reps 10 --kernels gram2 >> $O/gram_ab.jsonl 2>> $O/gram_ab.err
  step "ab_base_$k" timeout -k 10 120 env GNK_LIB=tools/_diag/libgnk_base.so python tools/kbench.py --k $k --reps 10 --kernels gram2 | sed 's/^{/{"lib": "base", /' >> $O/gram_ab.jsonl 2>> $O/gram_ab.err
done
step bench timeout -k 10 600 python bench.py --warmup 5 --cpu-seconds 0 --cg-iters 0 > $O/bench.json 2> $O/bench.err
echo done
