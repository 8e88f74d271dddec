#!/bin/bash
# Per-dispatch kernel trace of a short bench (+ saved model for leaf sizes). TAG names the output dir.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out/trace_${TAG:-x}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench \
  -- python3 "$ROOT/bench.py" --steps 4 --warmup 1 --save-model "$OUT/model.txt" ${BENCH_ARGS} > "$OUT/stdout.log" 2>&1
echo "rocprof rc=$?"
