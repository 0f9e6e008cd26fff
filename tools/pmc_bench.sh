#!/bin/bash
# HBM traffic of the bench's dominant kernel: two rocprofv3 counter passes (FETCH_SIZE,
# WRITE_SIZE; --kernel-trace only) over the driver's bench command (its default steps, warmup and
# repeats), then tools/pmc_summary.py over exactly the timed regions' Gram launches (the
# window file bench.py writes).  Extra arguments go to bench.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/pmc_bench"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  GNK_BENCH_WINDOW_OUT="$OUT/window_$c.json" timeout -k 10 500 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$c" -o run --output-format csv -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --cg-iters 0 --jvp-reps 5 "$@" > "$OUT/$c.log" 2>&1 || exit $?
done
cmp -s <(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['gram_launch_offset'], d['launch_bytes'])" "$OUT/window_FETCH_SIZE.json") \
       <(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['gram_launch_offset'], d['launch_bytes'])" "$OUT/window_WRITE_SIZE.json") \
  || { echo "the two counter passes timed different Gram windows" >&2; exit 1; }
python3 "$R/tools/pmc_summary.py" "$OUT" "${PMC_CONFIG:-bratu8192_gnk_restart20_res_old_ranks1}" "$OUT/window_FETCH_SIZE.json" > "$OUT/pmc_summary.json"
