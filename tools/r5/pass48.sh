#!/bin/bash
# Round-5 pass 48: expansions per round (SML_GBDT_SPEC) at 63 / 127 / 255 leaves.
OUT=${1:-gpurun_out/r5p48}
mkdir -p "$OUT"
for L in 255 127 63; do
  for k in 4 8 16; do
    SML_GBDT_SPEC=$k timeout -k 10 300 python bench.py --steps 2 --warmup 1 --leaves $L > "$OUT/bench_L${L}_s$k.log" 2>&1 || exit 1
    echo "leaves $L spec $k: $(tail -1 "$OUT/bench_L${L}_s$k.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['iteration_ms'], round(d['config']['holdout_auc'], 5))")"
  done
done
