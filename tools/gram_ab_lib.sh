#!/bin/bash
# A/B of the product libgnk.so against tools/_var/libgnk_$1.so on the Gram pass: bit-identity and time
# per k (tools/gram_dump.py), interleaved twice.  Usage: tools/gram_ab_lib.sh VARIANT k1,k2,... [grid]
set -o pipefail
V=$1; KS=$2; GRID=${3:-8192}
O=gpurun_out/gram_ab_$V
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 tools/gram_dump.py $O new $KS --grid $GRID >> $O/times.jsonl || exit $?
  GNK_LIB=tools/_var/libgnk_$V.so timeout -k 10 300 python3 tools/gram_dump.py $O $V $KS --grid $GRID >> $O/times.jsonl || exit $?
done
python3 tools/gram_dump.py --compare $O new $V > $O/bits.jsonl
