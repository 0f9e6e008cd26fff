#!/bin/bash
# Round-5 CG matvec grid session: the fused CG iteration under the previous library (tools/_var/libgnk_head.so) and
# the product, interleaved twice, then the whole -m gpu suite on the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/cg_grid_ab.jsonl
for i in 1 2; do
  for lib in head prod; do
    if [[ $lib == prod ]]; then so=gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so; else so=tools/_var/libgnk_head.so; fi
    GNK_LIB=$so timeout -k 10 300 python tools/cg_ab.py | sed "s/^/{\"lib\": \"$lib\", \"res\": /; s/\$/}/" >> gpurun_out/cg_grid_ab.jsonl || exit 1
  done
done
grep device_lagged gpurun_out/cg_grid_ab.jsonl
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r5g.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu_r5g.log
