#!/bin/bash
# Round-5 single-reduction CG session: bit fingerprint vs tools/_var/libgnk_head.so, the CG / GN / generic tests,
# and the bench line (gn_cg incl. the single-reduction option).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_prod.npz || exit 1
GNK_LIB=tools/_var/libgnk_head.so timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_head.npz || exit 1
python tools/kernel_bits.py --compare /tmp/kb_prod.npz /tmp/kb_head.npz > gpurun_out/kb_sr.txt
grep -c identical gpurun_out/kb_sr.txt; grep -v identical gpurun_out/kb_sr.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_cg_device.py tests/test_gpu_generic.py tests/test_gpu_multislab.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/sr_tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/sr_tests.log
timeout -k 10 300 python bench.py --warmup 5 > gpurun_out/bench_r5h.json 2> gpurun_out/bench_r5h.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_r5h.json')); g=d['gn_cg']; print(d['value'], g['ms_per_iter'], g['single_reduction']['ms_per_iter'], g['matvec']['avg_launch_ms'])"
