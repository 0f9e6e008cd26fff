#!/bin/bash
# Round-5 pending-GEMV session: bit fingerprint vs the previous library (tools/_var/libgnk_head.so), the
# kernel's time (kbench gemvp), the C2 / baseline-size tests, and a whole-bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_prod.npz || exit 1
GNK_LIB=tools/_var/libgnk_head.so timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_head.npz || exit 1
python tools/kernel_bits.py --compare /tmp/kb_prod.npz /tmp/kb_head.npz | tee gpurun_out/kb_gemvp.txt | grep -v identical
rm -f gpurun_out/ab.jsonl
AB_LIBS="head prod" AB_KS="4 12 20" AB_KERNELS=gemvp AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh > /dev/null || exit $?
cat gpurun_out/ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline_sizes.py tests/test_gpu_kernels.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gemvp_tests.log 2>&1; tail -3 gpurun_out/gemvp_tests.log
rm -f gpurun_out/bench_ab.jsonl
AB_LIBS="head prod" AB_ROUNDS=3 timeout -k 10 900 bash tools/bench_ab.sh > /dev/null || exit $?
python3 -c "
import json
for l in open('gpurun_out/bench_ab.jsonl'):
    d=json.loads(l); print(d['lib'], d['round'], round(d['value'],1), round(d['gram_ms'],4), round(d['trial_ms'],4))"
