#!/bin/bash
# Round-5 wide vjp_gemv_t session: bit fingerprint vs tools/_var/libgnk_head.so (incl. k = 25..100), the
# basis / segment tests, kbench vjpg at k = 40 / 100 (16384^2) new vs head, then the capped C5 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5l
export TMPDIR=/tmp
if [[ -z "$SKIP_CHECKS" ]]; then
timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_prod.npz || exit 1
GNK_LIB=tools/_var/libgnk_head.so timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_head.npz || exit 1
python tools/kernel_bits.py --compare /tmp/kb_prod.npz /tmp/kb_head.npz > gpurun_out/r5l/kernel_bits.txt
grep -c identical gpurun_out/r5l/kernel_bits.txt; grep -v identical gpurun_out/r5l/kernel_bits.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_segments.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5l/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5l/pytest.log; [[ $rc == 0 ]] || exit $rc
fi
for i in 1 2; do
  for k in 40 100; do
    timeout -k 10 300 python3 tools/kbench.py --grid 16384 --k $k --reps 5 --kernels vjpg | sed "s/^/new k=$k /" || exit 1
    GNK_LIB=tools/_var/libgnk_head.so timeout -k 10 300 python3 tools/kbench.py --grid 16384 --k $k --reps 5 --kernels vjpg | sed "s/^/head k=$k /" || exit 1
  done
done
timeout -k 10 500 python3 bench.py --grid 16384 --restart 100 --steps 99 --warmup 1 --repeats 1 --cpu-seconds 0 --cg-iters 0 --jvp-reps 2 > gpurun_out/r5l/bench_c5.json 2> gpurun_out/r5l/bench_c5.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r5l/bench_c5.json')); print('C5', d['value'], d['ms_per_step'])"
