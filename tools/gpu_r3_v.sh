#!/bin/bash
# Round 3 profiles of the driver's bench command: rocprofv3 kernel trace + stats (and the timed window's
# Gram launches from it), then the FETCH_SIZE / WRITE_SIZE passes over the same window.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
echo "== rocprof $(date +%T)"
bash tools/rocprof_bench.sh || { echo "rocprof failed rc=$?"; exit 1; }
echo "== pmc $(date +%T)"
bash tools/pmc_bench.sh || { echo "pmc failed rc=$?"; exit 1; }
echo "done $(date +%T)"
