set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/fused_ab.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_kern.log 2>&1 || { echo KERNEL_TEST_FAIL; exit 1; }
FUSED_KS="9 11 13 15 17" bash tools/fused_ab.sh; echo "ab6 rc=$?"
mv gpurun_out/fused_ab.jsonl gpurun_out/fused_ab_r6.jsonl
GNK_FUSED_RING=5 FUSED_KS="11 15" bash tools/fused_ab.sh; echo "ab5 rc=$?"
