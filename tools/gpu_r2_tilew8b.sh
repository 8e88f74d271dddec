#!/bin/bash
# A/B: fp32 8-wave 64x128 / 128x64 tiles vs the default (8-wave 64x64), per layer; the new tiles' exactness test.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-tilew8b}
mkdir -p $OUT
for t in default 64x998 128x998; do
  if [ $t = default ]; then
    timeout -k 10 300 python tools/bench_conv.py --dtype fp32 --no-ref > $OUT/tile_fp32_$t.log 2>&1 || exit $?
  else
    SML_CONV_TILE=$t timeout -k 10 300 python tools/bench_conv.py --dtype fp32 --no-ref > $OUT/tile_fp32_$t.log 2>&1 || exit $?
  fi
  echo "fp32 $t $(tail -1 $OUT/tile_fp32_$t.log)"
done
