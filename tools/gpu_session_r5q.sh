#!/bin/bash
# Round-5: k_gram_x at 7 column blocks with RinvAug's B fragments read from LDS (no spill) vs
# tools/_var/libgnk_prev.so (B fragments in VGPRs, 112 B of spill per lane); Gram tests, then time per k.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5q
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gram" --timeout 300 --timeout-method thread > gpurun_out/r5q/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5q/pytest.log; [[ $rc == 0 ]] || exit $rc
O=gpurun_out/r5q/gram; rm -rf $O; mkdir -p $O
KS=80,96,100,111
for i in 1 2; do
  timeout -k 10 300 python3 tools/gram_dump.py $O new $KS >> $O/times.jsonl || exit $?
  GNK_LIB=tools/_var/libgnk_prev.so timeout -k 10 300 python3 tools/gram_dump.py $O prev $KS >> $O/times.jsonl || exit $?
done
python3 - <<'PY'
import json, collections, numpy as np
O = "gpurun_out/r5q/gram"
t = collections.defaultdict(list)
for l in open(O + "/times.jsonl"):
    d = json.loads(l); t[(d["k"], d["tag"])].append(d["ms"])
for k in sorted({k for k, _ in t}):
    A, B = np.load(f"{O}/G_new_k{k}.npy"), np.load(f"{O}/G_prev_k{k}.npy")
    print(f"k={k:4d} new {min(t[(k, 'new')]):8.3f} prev {min(t[(k, 'prev')]):8.3f} identical {np.array_equal(A, B)}")
PY
