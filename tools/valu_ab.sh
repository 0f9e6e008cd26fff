# A/B of the Gram-pass kernels at 8192^2 (VALU vs staged MFMA), plus the Gram tests
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gram" --timeout 120 > gpurun_out/valu_test.log 2>&1 || exit $?
rm -f gpurun_out/valu_bench.txt
for k in ${KS:-1 2 3 4 5 6 7 8}; do
  timeout -k 10 120 env GNK_GRAM_VALU=1 python tools/kbench.py --k $k --kernels gram2 >> gpurun_out/valu_bench.txt || exit $?
  timeout -k 10 120 env GNK_GRAM_VALU=0 python tools/kbench.py --k $k --kernels gram2 >> gpurun_out/valu_bench.txt || exit $?
done
