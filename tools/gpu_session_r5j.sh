#!/bin/bash
# Round-5 wide-Gram session 2: k_gram_x from 2 column blocks (GNK_TUNE_GRAM_WIDE 4) against the chunked /
# prefetching kernels (product default) and the round's head library, per k, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/gram_x_lo
rm -rf $O; mkdir -p $O
KS=${KS:-21,27,33,40,47,48,51,56,63}
for i in 1 2; do
  timeout -k 10 300 python3 tools/gram_dump.py $O dflt $KS >> $O/times.jsonl || exit $?
  timeout -k 10 300 python3 tools/gram_dump.py $O x $KS --tune gram_wide=4 >> $O/times.jsonl || exit $?
  GNK_LIB=tools/_var/libgnk_head.so timeout -k 10 300 python3 tools/gram_dump.py $O head $KS >> $O/times.jsonl || exit $?
done
python3 tools/gram_dump.py --compare $O dflt head > $O/bits_dflt_head.jsonl
python3 tools/gram_dump.py --compare $O x dflt > $O/bits_x_dflt.jsonl
grep -c true $O/bits_dflt_head.jsonl
python3 - <<'PY'
import json, collections, numpy as np, glob
O = "gpurun_out/gram_x_lo"
t = collections.defaultdict(list)
for l in open(O + "/times.jsonl"):
    d = json.loads(l); t[(d["k"], d["tag"])].append(d["ms"])
for k in sorted({k for k, _ in t}):
    print(f"k={k:4d} head {min(t[(k, 'head')]):8.3f} dflt {min(t[(k, 'dflt')]):8.3f} x {min(t[(k, 'x')]):8.3f}")
for l in open(O + "/bits_x_dflt.jsonl"):
    d = json.loads(l)
    A = np.load(f"{O}/G_dflt_k{d['k']}.npy")
    print(d["k"], "x vs dflt rel", d["max_abs_diff"] / np.max(np.abs(A)))
PY
