#!/bin/bash
# Where the staged Gram pass's wave cycles go (k = 12: one column block, two workgroups per CU; k = 17: two
# blocks, one workgroup): tools/pmc_sq.sh's two passes plus a third of issue / co-execution counters, each
# pass its own rocprofv3 run (--kernel-trace only, <= 8 SQ counters).  Usage: tools/pmc_sq_gram_s.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/r5/sqs}
R="${GRAFT_REPO_ROOT:-$(pwd)}"
for k in 12 17; do
  bash "$R/tools/pmc_sq.sh" "$OUT/k$k" --grid 8192 --k $k --reps 3 --kernels gram2 || exit $?
  ( cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU \
      SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_SALU \
      SQ_LDS_DATA_FIFO_FULL -d "$R/$OUT/k$k/p3" -o run --output-format csv -- \
      python3 "$R/tools/kbench.py" --grid 8192 --k $k --reps 3 --kernels gram2 > "$R/$OUT/k$k/p3.log" 2>&1 ) || exit $?
done
