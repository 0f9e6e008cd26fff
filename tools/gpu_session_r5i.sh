#!/bin/bash
# Round-5 wide-Gram session: the Gram pass per k (bits + time, interleaved twice) of the product library against
# tools/_var/libgnk_head.so -- the pair-tile index of the wide passes folded at compile time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/gram_ab_head
timeout -k 10 900 bash tools/gram_ab_lib.sh head ${KS:-5,12,20,21,33,40,47,48,51,63,64,70,80,96,100,111} > gpurun_out/ab_head.log 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/ab_head.log; exit 1; }
cat gpurun_out/gram_ab_head/bits.jsonl
python3 - <<'EOF'
import json, collections
t = collections.defaultdict(list)
for l in open("gpurun_out/gram_ab_head/times.jsonl"):
    d = json.loads(l); t[(d["k"], d["tag"])].append(d["ms"])
for k in sorted({k for k, _ in t}):
    n, h = min(t[(k, "new")]), min(t[(k, "head")])
    print(f"k={k:4d} new {n:8.3f} head {h:8.3f} ratio {n / h:.3f}")
EOF
