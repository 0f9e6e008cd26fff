#!/bin/bash
# Round 3: rehearsal of the bench's multi-rank path (torchrun, 2 ranks sharing the one MI355X, gloo with
# host-staged collectives -- the driver's N > 1 runs use RCCL, one GPU per rank).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3y
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 GNK_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node 2 bench.py --gpus 2 > $O/bench2.json 2> $O/bench2.err
echo "bench2 rc=$?"
