#!/bin/bash
# Round-5: 1024 blocks per chunk for the wide vjp_gemv_t (product) vs 2048 / nchunk (tools/_var/libgnk_prev.so);
# the segment / basis tests, kbench vjpg at 16384^2 interleaved twice, the capped C5 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5n
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5n/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5n/pytest.log; [[ $rc == 0 ]] || exit $rc
for i in 1 2; do
  for k in ${KS:-25 40 57 100}; do
    timeout -k 10 300 python3 tools/kbench.py --grid 16384 --k $k --reps 5 --kernels vjpg | sed "s/^/new k=$k /" || exit 1
    GNK_LIB=tools/_var/libgnk_prev.so timeout -k 10 300 python3 tools/kbench.py --grid 16384 --k $k --reps 5 --kernels vjpg | sed "s/^/prev k=$k /" || exit 1
  done
done
timeout -k 10 500 python3 bench.py --grid 16384 --restart 100 --steps 99 --warmup 1 --repeats 1 --cpu-seconds 0 --cg-iters 0 --jvp-reps 2 > gpurun_out/r5n/bench_c5.json 2> gpurun_out/r5n/bench_c5.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r5n/bench_c5.json')); print('C5', d['value'], d['ms_per_step'])"
