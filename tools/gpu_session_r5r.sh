#!/bin/bash
# Round-5: k_gram_w at 2 column blocks (k = 21..31) on 32-row chunks (tools/_var/libgnk_c32.so: 42 KB of LDS per
# workgroup, three per CU) vs the product's 64-row chunks (76 KB, two per CU), 8192^2, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5r; rm -rf $O; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 tools/gram_dump.py $O prod 21,24,27,31 >> $O/times.jsonl || exit $?
  GNK_LIB=tools/_var/libgnk_c32.so timeout -k 10 300 python3 tools/gram_dump.py $O c32 21,24,27,31 >> $O/times.jsonl || exit $?
done
python3 - <<'PY'
import json, collections, numpy as np
O = "gpurun_out/r5r"
t = collections.defaultdict(list)
for l in open(O + "/times.jsonl"):
    d = json.loads(l); t[(d["k"], d["tag"])].append(d["ms"])
for k in sorted({k for k, _ in t}):
    A, B = np.load(f"{O}/G_c32_k{k}.npy"), np.load(f"{O}/G_prod_k{k}.npy")
    print(f"k={k:4d} prod {min(t[(k, 'prod')]):8.3f} c32 {min(t[(k, 'c32')]):8.3f} rel {np.max(np.abs(A - B)) / np.max(np.abs(B)):.1e}")
PY
