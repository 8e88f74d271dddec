#!/bin/bash
# Kernel + memory-copy trace of the ONNXModel DataFrame path (fp16): GPU busy vs wall per batch.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT=$ROOT/gpurun_out/${TAG:-dpprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof -o dp \
  -- python3 $ROOT/tools/bench_onnx_dp.py --images 2048 --precisions fp16 > $OUT/stdout.log 2>&1
echo "rocprof rc=$?"
grep '^{' $OUT/stdout.log | cut -c1-160
