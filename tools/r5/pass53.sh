#!/bin/bash
# Round-5 pass 53: the replay's child reads in one LDS round trip: GBDT GPU tests, plan phases at 31 / 255
# leaves, fits.
OUT=${1:-gpurun_out/r5p53}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || { grep -E "FAILED" "$OUT/pytest_gbdt.log" | head; exit 1; }
tail -1 "$OUT/pytest_gbdt.log"
for L in 31 255; do
  SML_BPLAN_PROF=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --leaves $L > "$OUT/bench_prof_L$L.log" 2> "$OUT/phases_L$L.txt" || exit 1
  echo "L$L $(grep 'bplan phases' "$OUT/phases_L$L.txt" | tail -1)"
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --leaves $L > "$OUT/bench_L$L.log" 2>&1 || exit 1
  echo "leaves $L: $(tail -1 "$OUT/bench_L$L.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['iteration_ms'], round(d['config']['holdout_auc'], 5))")"
done
