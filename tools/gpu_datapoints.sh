#!/bin/bash
# Single-GPU data points of the other BASELINE configs (round 5): capped C5 (16384^2, restart 100, k = 2..100),
# the C4 grid on one GPU (32768^2, the first outer iterations, CGLS at that size), and the multi-rank bench
# rehearsal through bench.py's own launcher (2 gloo ranks sharing the GPU).  Each step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5
timeout -k 10 500 python3 bench.py --grid 16384 --restart 100 --steps 99 --warmup 1 --repeats 1 --cpu-seconds 0 --cg-iters 0 --jvp-reps 2 > gpurun_out/r5/bench_c5_capped.json 2> gpurun_out/r5/bench_c5_capped.err || exit $?
timeout -k 10 500 python3 bench.py --grid 32768 --steps 4 --warmup 1 --repeats 1 --cpu-seconds 0 --cg-iters 20 --jvp-reps 5 > gpurun_out/r5/bench_32768.json 2> gpurun_out/r5/bench_32768.err || exit $?
GNK_BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --cpu-seconds 0 --cg-iters 20 > gpurun_out/r5/bench_2rank_gloo.json 2> gpurun_out/r5/bench_2rank_gloo.err || exit $?
echo done
