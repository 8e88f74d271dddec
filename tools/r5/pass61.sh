#!/bin/bash
# Round-5 pass 61: host look-ahead of the batched rounds on the final code (SML_GBDT_LOOKAHEAD 1 = default, 2).
OUT=${1:-gpurun_out/r5p61}
mkdir -p "$OUT"
for k in 1 2 1 2; do
  SML_GBDT_LOOKAHEAD=$k timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$OUT/bench_look$k.log" 2>&1 || exit 1
  echo "lookahead $k: $(tail -1 "$OUT/bench_look$k.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'])")"
done
