#!/bin/bash
# Round 3, GPU session I: kernel parity (staged Gram: EB one-block-column, 5-slot two-block-column),
# the 8192^2 full restart cycle vs the pinned oracle, the multi-rank solver tests (RCCL-path shim,
# Dot2 pairs across ranks), the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3i
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
PYT="python -u -m pytest -x -v -s --timeout 900 --timeout-method thread"
step kernels timeout -k 10 300 $PYT tests/test_gpu_kernels.py > $O/kernels.log 2>&1
step cycle timeout -k 10 300 $PYT tests/test_gpu_baseline_sizes.py -k full_restart_cycle > $O/cycle.log 2>&1
step multislab timeout -k 10 600 $PYT tests/test_gpu_multislab.py > $O/multislab.log 2>&1
step bench timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
echo done
