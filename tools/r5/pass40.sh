#!/bin/bash
# Round-5 pass 40: lambdarank kernel time with and without the O(cnt^2) rank count (SML_RANK_PROF_PHASE=1:
# identity ranks, timing only).
OUT=${1:-gpurun_out/r5p40}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for v in 0 1; do
  ( export SML_RANK_PROF_PHASE=$v; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_$v.log" 2>&1 ) || exit 1
  f=$(find "$OUT/prof_$v" -name '*kernel_stats.csv' -print -quit)
  echo "phase $v"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "lambdarank" in r["Name"]:
        print(f'  {float(r["AverageNs"])/1e3:8.1f} us/call x {r["Calls"]}  {r["Name"][:70]}')
PY
  rm -rf "$OUT/prof_$v"
done
