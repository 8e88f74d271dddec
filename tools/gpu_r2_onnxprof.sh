#!/bin/bash
# Kernel trace of the ResNet-50 fp16 batch-128 session (per-kernel time by conv tile / prologue variant).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT=$ROOT/gpurun_out/${TAG:-onnxprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o onnx \
  -- python3 $ROOT/tools/bench_onnx.py --batches 128 --precisions ${PREC:-fp16} --iters 20 --images 0 > $OUT/prof_stdout.log 2>&1
echo "rocprof rc=$?"
grep '^{' $OUT/prof_stdout.log | head -3
