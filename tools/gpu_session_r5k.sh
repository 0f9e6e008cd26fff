#!/bin/bash
# Round-5 wide-Gram session 3: k_gram_x for 4..7 column blocks with the FMA stencil -- the Gram tests and the
# large-configuration (C5) tests, then time per k against the round's head library (interleaved twice).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large_configs.py tests/test_gpu_generic.py -m gpu -x -q --durations=8 --timeout 600 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -14 gpurun_out/pytest_wide.log; [[ $rc == 0 ]] || exit $rc
O=gpurun_out/gram_ab_head2
rm -rf $O; mkdir -p $O
KS=${KS:-47,48,51,56,63,64,70,80,96,100,111}
for i in 1 2; do
  timeout -k 10 300 python3 tools/gram_dump.py $O new $KS >> $O/times.jsonl || exit $?
  GNK_LIB=tools/_var/libgnk_head.so timeout -k 10 300 python3 tools/gram_dump.py $O head $KS >> $O/times.jsonl || exit $?
done
python3 - <<'PY'
import json, collections, numpy as np
O = "gpurun_out/gram_ab_head2"
t = collections.defaultdict(list)
for l in open(O + "/times.jsonl"):
    d = json.loads(l); t[(d["k"], d["tag"])].append(d["ms"])
for k in sorted({k for k, _ in t}):
    A, B = np.load(f"{O}/G_new_k{k}.npy"), np.load(f"{O}/G_head_k{k}.npy")
    n, h = min(t[(k, "new")]), min(t[(k, "head")])
    print(f"k={k:4d} new {n:8.3f} head {h:8.3f} ratio {n / h:.3f} rel_diff {np.max(np.abs(A - B)) / np.max(np.abs(B)):.2e}")
PY
