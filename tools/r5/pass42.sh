#!/bin/bash
# Round-5 pass 42: how often the previous iteration's rank order converges within 2 / 8 / 32 pass pairs.
OUT=${1:-gpurun_out/r5p42}
mkdir -p "$OUT"
for v in 2 8 32; do
  SML_RANK_OE_MAX=$v SML_RANK_OE_STATS=1 timeout -k 10 300 python tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/bench_oe$v.log" 2> "$OUT/oe$v.txt" || exit 1
  echo "oe_max $v: $(grep 'rank order reuse' "$OUT/oe$v.txt" | tail -1)"
done
