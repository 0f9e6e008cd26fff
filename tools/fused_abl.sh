#!/bin/bash
# fused-pass ablations (tools/abl_fused.sh builds): time of the pass with parts removed, 8192^2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/fused_abl.jsonl
for K in 11 13; do
  for m in 0 1 2 4 8 15; do
    lib=gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so
    [[ $m != 0 ]] && lib=tools/_ablf/libgnk_f$m.so
    echo -n "{\"mask\": $m, \"run\": " >> gpurun_out/fused_abl.jsonl
    GNK_LIB=$lib timeout -k 10 120 python tools/kbench.py --k $K --reps 10 --kernels fused,gram2n >> gpurun_out/fused_abl.jsonl 2>> gpurun_out/fused_abl.err || exit $?
    echo "}" >> gpurun_out/fused_abl.jsonl
  done
done
echo ok
