#!/bin/bash
# Gram-pass timing per basis size at 8192^2 (tools/kbench.py gram2: the preconditioned pass with r),
# after the GPU tests of the Gram kernels.  Usage: GRAM_KS="17 20" bash tools/gram_ab.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "gram" > gpurun_out/gram_tests.log 2>&1 || exit $?
: > gpurun_out/gram_ab.jsonl
for k in ${GRAM_KS:-9 12 16 17 20}; do
  timeout -k 10 120 python tools/kbench.py --k $k --reps 10 --kernels ${GRAM_KERNELS:-gram2} >> gpurun_out/gram_ab.jsonl 2>> gpurun_out/gram_ab.err || exit $?
done
