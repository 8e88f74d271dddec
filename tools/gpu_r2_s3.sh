#!/bin/bash
# Session-3 check: 8-wave 128x128 conv tile A/B (fp32 + fp16), then the full round-2 check (all GPU tests, benches).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-s3}
mkdir -p $OUT
for dt in fp32 fp16; do
  for t in 128x999 default; do
    if [ $t = default ]; then
      timeout -k 10 300 python tools/bench_conv.py --dtype $dt --no-ref > $OUT/tile_${dt}_$t.log 2>&1 || exit $?
    else
      SML_CONV_TILE=$t timeout -k 10 300 python tools/bench_conv.py --dtype $dt --no-ref > $OUT/tile_${dt}_$t.log 2>&1 || exit $?
    fi
    echo "$dt $t $(tail -1 $OUT/tile_${dt}_$t.log)"
  done
done
TAG=${TAG:-s3}/full bash tools/gpu_r2_full.sh
