#!/bin/bash
# Round-5 pass 60: expansions per batched round at the headline's 31 leaves (SML_GBDT_SPEC 3..6; default 4).
OUT=${1:-gpurun_out/r5p60}
mkdir -p "$OUT"
for k in 4 5 6 3 4; do
  SML_GBDT_SPEC=$k timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$OUT/bench_spec$k.log" 2>&1 || exit 1
  echo "spec $k: $(tail -1 "$OUT/bench_spec$k.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'])")"
done
