#!/bin/bash
# Round-5 pass 41: lambdarank ranks from the previous iteration's order (odd-even transposition passes, the
# count as fallback): ranking GPU tests, kernel table with and without (SML_RANK_OE_MAX=0), ranker bench.
OUT=${1:-gpurun_out/r5p41}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py -k "rank or lambda" > "$OUT/pytest_rank.log" 2>&1 || { grep -E "FAILED|Error" "$OUT/pytest_rank.log" | head -20; tail -5 "$OUT/pytest_rank.log"; exit 1; }
tail -1 "$OUT/pytest_rank.log"
for v in 8 0; do
  ( export SML_RANK_OE_MAX=$v; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_$v.log" 2>&1 ) || exit 1
  f=$(find "$OUT/prof_$v" -name '*kernel_stats.csv' -print -quit)
  echo "oe_max $v: $(tail -1 "$OUT/prof_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ndcg@10_holdout_slice'))")"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "lambdarank" in r["Name"]:
        print(f'  {float(r["AverageNs"])/1e3:8.1f} us/call x {r["Calls"]}  {r["Name"][:70]}')
PY
  rm -rf "$OUT/prof_$v"
done
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
tail -1 "$OUT/bench_ranker.log" | cut -c1-300
