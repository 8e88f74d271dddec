#!/bin/bash
# Round-5 pass 29: speculation waste per tree (SML_BPLAN_PROF) and the fit at 3 / 4 / 5 expansions per round.
OUT=${1:-gpurun_out/r5p29}
mkdir -p "$OUT"
for k in 4 3 5 6; do
  SML_GBDT_SPEC=$k SML_BPLAN_PROF=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 > "$OUT/bench_prof_spec$k.log" 2> "$OUT/bplan_spec$k.txt" || exit 1
  echo "spec $k"; tail -2 "$OUT/bplan_spec$k.txt"
done
for k in 3 4 5 4 3 5; do
  SML_GBDT_SPEC=$k timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$OUT/bench_spec$k.log" 2>&1 || exit 1
  echo "spec $k $(grep -o '"iteration_ms": [0-9.]*' "$OUT/bench_spec$k.log")"
done
