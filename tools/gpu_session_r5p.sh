#!/bin/bash
# Round-5: k_gram_x from 3 column blocks, two workgroups per CU at 2..4 blocks -- the Gram / large-config tests,
# the Gram pass per k against tools/_var/libgnk_prev.so (interleaved twice), the capped C5 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r5p
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large_configs.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r5p/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r5p/pytest.log; [[ $rc == 0 ]] || exit $rc
O=gpurun_out/r5p/gram; rm -rf $O; mkdir -p $O
KS=31,32,33,40,47,48,56,63
for i in 1 2; do
  timeout -k 10 300 python3 tools/gram_dump.py $O new $KS >> $O/times.jsonl || exit $?
  GNK_LIB=tools/_var/libgnk_prev.so timeout -k 10 300 python3 tools/gram_dump.py $O prev $KS >> $O/times.jsonl || exit $?
done
python3 - <<'PY'
import json, collections, numpy as np
O = "gpurun_out/r5p/gram"
t = collections.defaultdict(list)
for l in open(O + "/times.jsonl"):
    d = json.loads(l); t[(d["k"], d["tag"])].append(d["ms"])
for k in sorted({k for k, _ in t}):
    A, B = np.load(f"{O}/G_new_k{k}.npy"), np.load(f"{O}/G_prev_k{k}.npy")
    print(f"k={k:4d} new {min(t[(k, 'new')]):8.3f} prev {min(t[(k, 'prev')]):8.3f} rel_diff {np.max(np.abs(A - B)) / np.max(np.abs(B)):.2e}")
PY
timeout -k 10 500 python3 bench.py --grid 16384 --restart 100 --steps 99 --warmup 1 --repeats 1 --cpu-seconds 0 --cg-iters 0 --jvp-reps 2 > gpurun_out/r5p/bench_c5.json 2> gpurun_out/r5p/bench_c5.err || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r5p/bench_c5.json')); print('C5', d['value'], d['ms_per_step'])"
