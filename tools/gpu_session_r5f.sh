#!/bin/bash
# Round-5 streaming-kernel session: bit fingerprint vs tools/_var/libgnk_head.so, the whole -m gpu suite, the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_prod.npz || exit 1
GNK_LIB=tools/_var/libgnk_head.so timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_head.npz || exit 1
python tools/kernel_bits.py --compare /tmp/kb_prod.npz /tmp/kb_head.npz > gpurun_out/kb_stream.txt
grep -c identical gpurun_out/kb_stream.txt; grep -v identical gpurun_out/kb_stream.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r5f.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu_r5f.log
timeout -k 10 300 python bench.py --warmup 5 > gpurun_out/bench_r5f.json 2> gpurun_out/bench_r5f.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r5f.json')); print(d['value'], d['ms_per_step'], d.get('cg'))"
