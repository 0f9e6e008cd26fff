set -o pipefail
for k in 64 80 100; do
  bash tools/pmc_sq.sh gpurun_out/r5/sqx_k$k --grid 8192 --k $k --reps 3 --kernels gram2 || exit $?
done
