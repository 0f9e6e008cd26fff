# Gram-pass tests + per-k timing at 8192^2 (tooling)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gram" --timeout 120 > gpurun_out/gk_test.log 2>&1 || exit $?
rm -f gpurun_out/gk_bench.txt
for k in ${KS:-13 14 16 17 18 20}; do
  timeout -k 10 120 python tools/kbench.py --k $k --kernels gram2 >> gpurun_out/gk_bench.txt || exit $?
done
