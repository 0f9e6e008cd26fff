# Prefetching wide-basis Gram (k_gram_wp, default for NB = 4) vs k_gram_w at 8192^2, plus the Gram
# tests with k_gram_wp forced for NB = 2, 3 as well (GNK_GRAM_WP=2).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gram" > gpurun_out/wp_test.log 2>&1 || exit $?
echo "== GNK_GRAM_WP=2" >> gpurun_out/wp_test.log
timeout -k 10 200 env GNK_GRAM_WP=2 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "test_gram_mfma and default" >> gpurun_out/wp_test.log 2>&1 || exit $?
rm -f gpurun_out/wp_ab.txt
for k in ${KS:-21 33 47 51 61}; do
  for e in "GNK_GRAM_WP=0" "GNK_GRAM_WP=1" "GNK_GRAM_WP=2"; do
    echo -n "k=$k $e " >> gpurun_out/wp_ab.txt
    timeout -k 10 120 env $e python tools/kbench.py --k $k --reps 5 --kernels gram1,gram2 >> gpurun_out/wp_ab.txt || exit $?
  done
done
