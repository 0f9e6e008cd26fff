#!/bin/bash
# Round-5 late session: the counter list, the k_gram_v1 DPP-neighbour A/B (library variant), then the
# round-end checks (tools/gpu_final.sh without the C5 point).  Each GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
rm -rf gpurun_out/gram_ab_dpp
timeout -k 10 400 bash tools/gram_ab_lib.sh dpp 8,9 > gpurun_out/ab_dpp.log 2>&1 || { echo AB_FAIL; exit 1; }
cat gpurun_out/gram_ab_dpp/bits.jsonl gpurun_out/gram_ab_dpp/times.jsonl
C5=0 bash tools/gpu_final.sh
