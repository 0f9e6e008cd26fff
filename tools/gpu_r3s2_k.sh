#!/bin/bash
# Round 3, session 2, GPU session K: the driver's bench command and smoke at the final commit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3s2k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
echo "done $(date +%T)"
