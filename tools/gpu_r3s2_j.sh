#!/bin/bash
# Round 3, session 2, GPU session J: single-GPU data points at the final kernels -- the C4 grid
# (32768^2, first 5 outer iterations, CGLS capped at 20) and the capped C5 (16384^2, restart 100, k to 100).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --grid 32768 --steps 4 --repeats 1 --cg-iters 20 --cpu-seconds 0 > $O/bench_32768.json 2> $O/bench_32768.err || exit $?
echo "32768 ok $(date +%T)"
timeout -k 10 600 python -u bench.py --grid 16384 --restart 100 --steps 99 --warmup 1 --repeats 1 --cpu-seconds 0 --cg-iters 0 --jvp-reps 2 > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
echo "done $(date +%T)"
