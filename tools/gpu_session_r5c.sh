#!/bin/bash
# Round-5 DPP lane-shift session: the -m gpu suite on the product library, then interleaved A/Bs against
# the previous library (tools/_var/libgnk_head.so): VALU Gram passes k = 1..9 (bits + time) and the whole bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_dpp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_dpp.log; [[ $rc == 0 ]] || exit $rc
rm -rf gpurun_out/gram_ab_head
timeout -k 10 400 bash tools/gram_ab_lib.sh head 1,3,5,7,8,9 > gpurun_out/ab_head.log 2>&1 || { echo AB_FAIL; exit 1; }
cat gpurun_out/gram_ab_head/bits.jsonl gpurun_out/gram_ab_head/times.jsonl
rm -f gpurun_out/bench_ab.jsonl
AB_LIBS="head prod" AB_ROUNDS=3 timeout -k 10 900 bash tools/bench_ab.sh || exit $?
bash tools/pmc_sq_gram_s.sh gpurun_out/r5/sqs || exit $?
