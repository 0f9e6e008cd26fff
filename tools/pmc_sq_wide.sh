#!/bin/bash
# SQ stall / pipe counters of the wide Gram passes (tools/pmc_sq.sh over kbench gram2 at 8192^2), one
# directory per k.  Usage: KS="33 51 64 80 100" tools/pmc_sq_wide.sh [OUTDIR]
set -o pipefail
OUT=${1:-gpurun_out/r5/sqx}
for k in ${KS:-64 80 100}; do
  bash tools/pmc_sq.sh $OUT/k$k --grid 8192 --k $k --reps 3 --kernels gram2 || exit $?
done
