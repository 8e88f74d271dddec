#!/bin/bash
# Round-5 pass 18: VW accuracy flake probe (staging pipeline on / off, device / host scoring, repeated), then the
# rest of pass 17 (VW bench, headline bench, ranker bench).
OUT=${1:-gpurun_out/r5p18}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 python tools/r5/vw_flake_probe.py 8 > "$OUT/vw_flake_probe.log" 2>&1 || { tail -20 "$OUT/vw_flake_probe.log"; exit 1; }
cat "$OUT/vw_flake_probe.log" | grep rep=
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
tail -1 "$OUT/bench_vw_estimator.log"
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
tail -1 "$OUT/bench_ranker.log" | cut -c1-300
