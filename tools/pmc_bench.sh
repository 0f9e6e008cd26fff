#!/bin/bash
# HBM traffic of the bench's dominant kernel: two rocprofv3 counter passes (FETCH_SIZE,
# WRITE_SIZE; --kernel-trace only) over a short bench run, then tools/pmc_summary.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/pmc_bench"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$c" -o run --output-format csv -- python3 "$R/bench.py" --cpu-seconds 0 --jvp-reps 5 "$@" > "$OUT/$c.log" 2>&1 || exit $?
done
python3 "$R/tools/pmc_summary.py" "$OUT" "${PMC_CONFIG:-bratu8192_gnk_restart20_res_old_ranks1}" > "$OUT/pmc_summary.json"
