#!/bin/bash
# Round-6 pass 25: kernel stats of the ResNet-50 v2 session, fp16 and fp32 at batch 256.
OUT=${1:-gpurun_out/r6p25}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for pr in fp16 fp32; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$pr" -o onnx -- python3 tools/bench_onnx.py --batches 256 --precisions $pr --iters 20 --images 256 > "$OUT/bench_$pr.log" 2>&1 || exit 1
  f=$(find "$OUT/prof_$pr" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_$pr.csv"
done
