#!/bin/bash
# One parameterised GPU-box session (replaces the per-session tools/gpu_session_r5*.sh scripts).
#   tools/gpu_session.sh TAG "PYTEST_ARGS" [BENCH_ARGS|-] [prof]
# Runs (each step under its own time limit, the chain stops at the first failure):
#   pytest PYTEST_ARGS (skipped when "-"), bench.py BENCH_ARGS (skipped when "-", no arguments when
#   "default"), and with "prof" the same
#   bench command under rocprofv3 --kernel-trace --stats.  Output: gpurun_out/TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; PYT=${2:--}; BARGS=${3:--}; PROF=${4:-}
O=gpurun_out/$TAG; rm -rf "$O"; mkdir -p "$O"
echo "== $TAG $(date +%T)"
if [[ "$PYT" != "-" ]]; then
  timeout -k 10 900 python -u -m pytest $PYT -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
[[ "$BARGS" == "default" ]] && BARGS=""
if [[ "$3" != "-" && -n "$3" ]]; then
  timeout -k 10 600 python bench.py $BARGS > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
  echo "bench ok"
fi
if [[ "$PROF" == "prof" && "$3" != "-" ]]; then
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $BARGS > "$GRAFT_REPO_ROOT/$O/bench_prof.json" 2> "$GRAFT_REPO_ROOT/$O/prof.err") || exit 1
  echo "prof ok"
fi
echo "== done $(date +%T)"
