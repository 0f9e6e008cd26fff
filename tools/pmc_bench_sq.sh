#!/bin/bash
# fp64 pipe use of the bench's Gram passes: one rocprofv3 counter pass (7 SQ + 1 GRBM
# counters, --kernel-trace only) over the driver's bench command, then tools/pmc_sq_summary.py over
# exactly the timed regions' Gram launches (the window file bench.py writes), per basis size k.
# Extra arguments go to bench.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/pmc_bench_sq"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTR="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
GNK_BENCH_WINDOW_OUT="$OUT/window.json" timeout -s KILL 600 rocprofv3 --kernel-trace --pmc $CTR -d "$OUT/sq" -o run --output-format csv -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --cg-iters 0 --jvp-reps 5 "$@" > "$OUT/sq.log" 2>&1 || exit $?
python3 "$R/tools/pmc_sq_summary.py" "$OUT/sq" "${PMC_CONFIG:-bratu8192_gnk_restart20_res_old_ranks1}" "$OUT/window.json" > "$OUT/pmc_sq_summary.json"
