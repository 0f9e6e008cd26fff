# VALU Gram: one-point-per-lane form (k = 7..9) vs the two-point form / staged kernel (tooling)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gram" --timeout 120 > gpurun_out/v1_test.log 2>&1 || exit $?
rm -f gpurun_out/v1_bench.txt
for k in 9 10; do
  for v in 1 0; do
    echo -n "V1=$v " >> gpurun_out/v1_bench.txt
    timeout -k 10 120 env GNK_GRAM_V1=$v python tools/kbench.py --k $k --kernels gram2 >> gpurun_out/v1_bench.txt || exit $?
  done
done
