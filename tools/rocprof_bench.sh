#!/bin/bash
# rocprofv3 kernel trace + stats of the driver's bench command (bench.py --gpus 1, its defaults),
# and the timed window's Gram launches averaged from the trace (tools/rocprof_window.py), to compare with
# the bench line's roofline.avg_launch_ms of the same run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/prof_bench"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
GNK_BENCH_WINDOW_OUT="$OUT/window.json" timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 "$R/tools/rocprof_window.py" "$(ls "$OUT"/*kernel_trace.csv "$OUT"/*/*kernel_trace.csv 2>/dev/null | head -1)" "$OUT/window.json" > "$OUT/window_avg.json"
