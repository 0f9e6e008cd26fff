#!/bin/bash
# Round 3, GPU session X (round-end check): the multi-rank solver tests (RCCL-path shim, Dot2 pairs across ranks), workers'
# progress streamed under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3x
mkdir -p $O
export TMPDIR=/tmp GNK_TEST_LOG_DIR=$PWD/$O/workers
step() {
  local name=$1; shift
  echo "== $name $(date +%T)"
  "$@"; local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  if [ $rc -ge 124 ]; then echo "FATAL at $name"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -x -v -s --timeout 900 --timeout-method thread"
step multislab timeout -k 10 1000 $PYT tests/test_gpu_multislab.py > $O/multislab.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err; echo "bench rc=$?"
echo done
