#!/bin/bash
# rocprofv3 counter passes (one counter group per pass; --kernel-trace only, no tracing
# domains) on the per-kernel microbenchmark.  Usage: tools/pmc.sh OUTDIR "kbench args"
set -o pipefail
OUT=$1; shift
ARGS="$*"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/$OUT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$R/$OUT/p$i" -o run --output-format csv -- python3 "$R/tools/kbench.py" $ARGS > "$R/$OUT/p$i.log" 2>&1 || exit $?
done
