#!/bin/bash
# Round-5 pass 59 (final code state): the bench's multi-rank launcher rehearsed with 2 and 4 ranks sharing the
# one GPU (exact int64 allreduce, P2P / RCCL data plane), then the 1-GPU headline once more.
OUT=${1:-gpurun_out/r5p59}
mkdir -p "$OUT"
timeout -k 10 500 python bench.py --gpus 2 --allow-shared-device --steps 2 --warmup 1 > "$OUT/bench_2rank_shared.log" 2>&1 || exit 1
tail -1 "$OUT/bench_2rank_shared.log"
timeout -k 10 600 python bench.py --gpus 4 --allow-shared-device --steps 2 --warmup 1 > "$OUT/bench_4rank_shared.log" 2>&1 || exit 1
tail -1 "$OUT/bench_4rank_shared.log"
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_1.log" 2>&1 || exit 1
tail -1 "$OUT/bench_1.log"
