#!/bin/bash
# Round-5 CG kernel session: bit fingerprint (operator, basis, Gram, CG kernels) vs the previous library
# (tools/_var/libgnk_head.so), the fused CG iteration's time under both libraries, and the CG / GN / generic tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_prod.npz || exit 1
GNK_LIB=tools/_var/libgnk_head.so timeout -k 10 200 python tools/kernel_bits.py /tmp/kb_head.npz || exit 1
python tools/kernel_bits.py --compare /tmp/kb_prod.npz /tmp/kb_head.npz > gpurun_out/kb_cg.txt
grep -c identical gpurun_out/kb_cg.txt; grep -v identical gpurun_out/kb_cg.txt
rm -f gpurun_out/cg_lib_ab.jsonl
for i in 1 2; do
  for lib in head prod; do
    if [[ $lib == prod ]]; then so=gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so; else so=tools/_var/libgnk_head.so; fi
    GNK_LIB=$so timeout -k 10 300 python tools/cg_ab.py | sed "s/^/{\"lib\": \"$lib\", \"res\": /; s/\$/}/" >> gpurun_out/cg_lib_ab.jsonl || exit 1
  done
done
cat gpurun_out/cg_lib_ab.jsonl
timeout -k 10 900 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_cg_device.py tests/test_gpu_generic.py tests/test_gpu_baseline_sizes.py tests/test_gpu_multislab.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/cg_tests.log 2>&1; tail -3 gpurun_out/cg_tests.log
