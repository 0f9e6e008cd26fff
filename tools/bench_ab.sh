#!/bin/bash
# Interleaved whole-bench A/B of library builds on one box ("prod" = the product library, NAME =
# tools/_var/libgnk_NAME.so).  Usage: AB_LIBS="head prod" AB_ROUNDS=2 bash tools/bench_ab.sh [bench args]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/bench_ab.jsonl"
mkdir -p "$R/gpurun_out"
for round in $(seq ${AB_ROUNDS:-2}); do
  for lib in ${AB_LIBS:-head prod}; do
    if [[ $lib == prod ]]; then so="$R/gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so"; else so="$R/tools/_var/libgnk_$lib.so"; fi
    GNK_LIB="$so" timeout -k 10 300 python "$R/bench.py" --cpu-seconds 0 --cg-iters 0 --jvp-reps 2 "$@" > "$R/gpurun_out/bench_ab_cur.json" 2>> "$R/gpurun_out/bench_ab.err" || exit $?
    python3 - "$lib" "$round" "$R/gpurun_out/bench_ab_cur.json" <<'PY' | tee -a "$OUT"
import json, sys
d = json.load(open(sys.argv[3]))
rf = d["roofline"]
print(json.dumps({"lib": sys.argv[1], "round": int(sys.argv[2]), "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "repeats": d.get("repeats"), "gram_ms": rf["avg_launch_ms"], "trial_ms": rf["trial"]["avg_launch_ms"],
                  "gram_by_k": {k: v["ms"] for k, v in rf["by_k"].items()}}))
PY
  done
done
