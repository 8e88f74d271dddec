#!/bin/bash
# Round-5 pass 45: one-shot P2P allreduce at the batched round's message size (2 ranks sharing the GPU), and the
# GBDT GPU tests on the final kernels.
OUT=${1:-gpurun_out/r5p45}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29541 tools/p2p_check.py > "$OUT/p2p_check_2rank_1gpu.log" 2>&1 || { tail -20 "$OUT/p2p_check_2rank_1gpu.log"; exit 1; }
grep -h '"rank"' "$OUT/p2p_check_2rank_1gpu.log" | cut -c1-400
timeout -k 10 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py tests/test_comm_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || { grep -E "FAILED" "$OUT/pytest_gbdt.log" | head; exit 1; }
tail -1 "$OUT/pytest_gbdt.log"
