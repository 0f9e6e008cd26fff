#!/bin/bash
# Round 3, GPU session W: k_gram_x transform with two accumulator chains per block (variant build in
# tools/_var, tools/build_variants.py gx2acc) vs the product build, 8192^2, k = 64 / 80 / 100.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3w
mkdir -p $O
for k in 64 80 100; do
  for lib in product gx2acc; do
    L=$PWD/gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so
    [ $lib != product ] && L=$PWD/tools/_var/libgnk_$lib.so
    GNK_LIB=$L timeout -k 10 150 python -u tools/kbench.py --k $k --reps 5 --kernels gram2 > $O/${lib}_$k.json || { echo "fail $lib $k"; exit 1; }
  done
done
echo done
