#!/bin/bash
# A/B of the product libgnk.so against a variant build (GNK_LIB) on the Gram pass: bit-identity of G and the
# median time per basis size, interleaved twice.  Usage (on the GPU box):
#   bash tools/lib_ab.sh TAG VARIANT_SO "k1,k2,..." [GRID]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; VAR=${2:?variant .so}; KS=${3:?ks}; GRID=${4:-8192}
O=gpurun_out/$TAG; rm -rf "$O"; mkdir -p "$O"
for i in 1 2; do
  timeout -k 10 300 python3 tools/gram_dump.py $O prod $KS --grid $GRID >> $O/times.jsonl || exit $?
  GNK_LIB=$VAR timeout -k 10 300 python3 tools/gram_dump.py $O var $KS --grid $GRID >> $O/times.jsonl || exit $?
done
python3 tools/gram_dump.py --compare $O prod var > $O/bits.jsonl
python3 - "$O" <<'PY'
import json, sys, collections
O = sys.argv[1]
t = collections.defaultdict(list)
for l in open(O + "/times.jsonl"):
    d = json.loads(l); t[(d["k"], d["tag"])].append(d["ms"])
bits = {json.loads(l)["k"]: json.loads(l)["bit_identical"] for l in open(O + "/bits.jsonl")}
for k in sorted({k for k, _ in t}):
    print(f"k={k:4d} prod {min(t[(k, 'prod')]):8.3f} var {min(t[(k, 'var')]):8.3f} bits_identical {bits.get(k)}")
PY
