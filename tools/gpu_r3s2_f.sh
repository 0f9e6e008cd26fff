#!/bin/bash
# Round 3, session 2, GPU session F: k_jvp2 (two grid rows per lane pass) -- the JVP kernel tests on the
# variant build, then the A/B vs the product build interleaved twice at 8192^2 and 16384^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2f
mkdir -p $O
export TMPDIR=/tmp
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  "$@"; local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  if [ $rc -ge 124 ]; then echo "FATAL at $name"; exit $rc; fi
  return 0
}
kb() {   # kb LIBTAG GRID
  local lib=$PWD/gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so
  [ "$1" != new ] && lib=$PWD/tools/_var/libgnk_$1.so
  GNK_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --grid $2 --k 4 --reps 30 --kernels jvp | sed "s/^/{\"lib\": \"$1\", \"r\": /; s/$/}/"
}
GNK_LIB=$PWD/tools/_var/libgnk_jvp2r.so step tests timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_solvers.py -k "jvp or gn" > $O/tests_jvp2r.log 2>&1
tail -3 $O/tests_jvp2r.log
for rep in 1 2; do
  for g in 8192 16384; do
    for v in new jvp2r; do
      step "jvp_${v}_${g}_$rep" kb $v $g >> $O/jvp2_ab.jsonl
    done
  done
done
echo done
