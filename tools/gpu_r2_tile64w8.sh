#!/bin/bash
# A/B: 64x64 tile with 8 waves (kernel=64999) vs the default table, fp16 and fp32, per layer.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-tile64w8}
mkdir -p $OUT
for dt in fp16 fp32; do
  for t in default 64x999 default2; do
    if [ $t = 64x999 ]; then
      SML_CONV_TILE=$t timeout -k 10 300 python tools/bench_conv.py --dtype $dt --no-ref > $OUT/tile_${dt}_$t.log 2>&1 || exit $?
    else
      timeout -k 10 300 python tools/bench_conv.py --dtype $dt --no-ref > $OUT/tile_${dt}_$t.log 2>&1 || exit $?
    fi
    echo "$dt $t $(tail -1 $OUT/tile_${dt}_$t.log)"
  done
done
