#!/bin/bash
# fused first trial + next Gram pass vs the unfused kernels it replaces (8192^2), per k
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for K in ${FUSED_KS:-9 11 12 13 15 16 17 19}; do
  timeout -k 10 120 python tools/kbench.py --k $K --reps 10 --kernels fused,gram2n,trialp,resid >> gpurun_out/fused_ab.jsonl 2>> gpurun_out/fused_ab.err || exit $?
done
