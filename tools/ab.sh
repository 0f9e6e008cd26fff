#!/bin/bash
# Interleaved A/B of variant builds (tools/build_variants.py -> tools/_var/libgnk_NAME.so; "prod" = the
# product library) on tools/kbench.py kernels.  Usage:
#   AB_LIBS="prod tv1" AB_KS="5 10 20" AB_KERNELS=trialp AB_ROUNDS=2 bash tools/ab.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$R/gpurun_out/ab.jsonl"
mkdir -p "$R/gpurun_out"
for round in $(seq ${AB_ROUNDS:-2}); do
  for k in ${AB_KS:-5 10 15 20}; do
    for lib in ${AB_LIBS:-prod}; do
      if [[ $lib == prod ]]; then so="$R/gauss_newton_via_generalized_krylov_subspaces_amd/libgnk.so"; else so="$R/tools/_var/libgnk_$lib.so"; fi
      line=$(GNK_LIB="$so" timeout -k 10 120 python "$R/tools/kbench.py" --grid ${AB_GRID:-8192} --k $k --reps ${AB_REPS:-10} --kernels ${AB_KERNELS:-trialp} ${AB_TUNE:+--tune $AB_TUNE} 2>> "$R/gpurun_out/ab.err") || exit $?
      echo "{\"lib\": \"$lib\", \"round\": $round, \"res\": $line}" | tee -a "$OUT"
    done
  done
done
