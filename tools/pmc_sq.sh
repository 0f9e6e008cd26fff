#!/bin/bash
# SQ stall / pipe counters (one pass, --kernel-trace only) on kbench.  Usage: tools/pmc_sq.sh OUTDIR "kbench args"
set -o pipefail
OUT=$1; shift
ARGS="$*"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/$OUT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$R/$OUT/p$i" -o run --output-format csv -- python3 "$R/tools/kbench.py" $ARGS > "$R/$OUT/p$i.log" 2>&1 || exit $?
done
