#!/bin/bash
# Round-5: k_gram_x at 4 waves per SIMD (two 8-wave workgroups per CU, amdgpu_waves_per_eu(4): 128 VGPRs, spills)
# vs the product (one workgroup per CU), 8192^2, 3 and 4 column blocks, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/gram_lb2; rm -rf $O; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 tools/gram_dump.py $O prod 33,47,51,63,64 --tune gram_wide=4 >> $O/times.jsonl || exit $?
  GNK_LIB=tools/_var/libgnk_lb2.so timeout -k 10 300 python3 tools/gram_dump.py $O lb2 33,47,51,63,64 --tune gram_wide=4 >> $O/times.jsonl || exit $?
done
cat $O/times.jsonl
