set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/fused_ab.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused_kern.log 2>&1 || { echo KERNEL_TEST_FAIL; exit 1; }
bash tools/fused_ab.sh; echo "ab rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline_sizes.py tests/test_mispredict.py -q -s --timeout 300 --timeout-method thread > gpurun_out/fused_e2e.log 2>&1; echo "e2e rc=$?"
timeout -k 10 300 python bench.py --cpu-seconds 0 --cg-iters 0 --jvp-reps 5 > gpurun_out/bench_fuse.json 2> gpurun_out/bench_fuse.err; echo "b1 rc=$?"
