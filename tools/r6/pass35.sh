#!/bin/bash
# Round-6 pass 35 (rebuilt extensions after the container re-creation): full GPU suite, smoke, headline
# bench, then the fp32 ResNet-50 session's kernel stats at batch 256.
OUT=${1:-gpurun_out/r6p35}
ROOT=$(pwd)
mkdir -p "$OUT"
bash tools/r6/full_gpu.sh "$OUT" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fp32" -o onnx -- python3 tools/bench_onnx.py --batches 256 --precisions fp32 --iters 20 --images 256 > "$OUT/bench_fp32.log" 2>&1 || exit 1
f=$(find "$OUT/prof_fp32" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_fp32.csv"
tail -3 "$OUT/bench_fp32.log"
