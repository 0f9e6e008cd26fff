# A/B of the staged Gram kernel's ring depth / blocks per CU at 8192^2 (tooling)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gram" --timeout 120 > gpurun_out/ring_test.log 2>&1 || exit $?
rm -f gpurun_out/ring_bench.txt
for k in ${KS:-9 10 12 13 14 16 17 18 20}; do
  for cfg in "default" "GNK_GRAM_RING=5" "GNK_GRAM_WG=1" "GNK_GRAM_RING=6 GNK_GRAM_WG=1"; do
    e=""; [ "$cfg" != default ] && e="$cfg"
    echo -n "$k $cfg " >> gpurun_out/ring_bench.txt
    timeout -k 10 120 env $e python tools/kbench.py --k $k --kernels gram2 >> gpurun_out/ring_bench.txt || exit $?
  done
done
