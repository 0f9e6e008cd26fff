#!/bin/bash
# Round-end measurement session: the driver's bench command, its rocprofv3 kernel stats (window
# Gram launches), and the window-matched PMC traffic (two counter passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --warmup 5 > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo BENCH_FAIL; exit 1; }
bash tools/rocprof_bench.sh || { echo ROCPROF_FAIL; exit 1; }
bash tools/pmc_bench.sh || { echo PMC_FAIL; exit 1; }
echo done
