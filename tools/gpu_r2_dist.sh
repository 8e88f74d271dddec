#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: 2 ranks share the device (gloo control
# plane + one-shot IPC histogram allreduce), vs the 1-rank run on the same per-rank rows.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/dist
mkdir -p $OUT
export PYTHONUNBUFFERED=1 MASTER_ADDR=127.0.0.1 HSA_ENABLE_IPC_MODE_LEGACY=0
ROWS=${ROWS:-2000000}
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --rows $ROWS > $OUT/n1.log 2>&1 || exit $?
tail -1 $OUT/n1.log | cut -c1-400
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29581 bench.py --gpus 2 --steps 10 --warmup 3 --rows $ROWS > $OUT/n2.log 2>&1 || exit $?
grep metric $OUT/n2.log | cut -c1-700
