#!/bin/bash
# Capped C5 (16384^2, restart 100, k = 2..100) bench line, then the same command under rocprofv3 --kernel-trace
# --stats (per-kernel totals of the whole run, to split the step's non-Gram time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/r5c5
ARGS="--grid 16384 --restart 100 --steps 99 --warmup 1 --repeats 1 --cpu-seconds 0 --cg-iters 0 --jvp-reps 2"
timeout -k 10 500 python3 bench.py $ARGS > gpurun_out/r5c5/bench.json 2> gpurun_out/r5c5/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5c5/prof" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/r5c5/bench_prof.json" 2> "$R/gpurun_out/r5c5/bench_prof.err" || exit $?
echo done
