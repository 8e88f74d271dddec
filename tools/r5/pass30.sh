#!/bin/bash
# Round-5 pass 30: ranker fit and its kernel table on the current GBDT kernels.
OUT=${1:-gpurun_out/r5p30}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rank" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_rank.log" 2>&1 || exit 1
f=$(find "$OUT/prof_rank" -name '*kernel_stats.csv' -print -quit)
python3 - "$f" > "$OUT/ranker_kernel_stats.txt" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f'{float(r["TotalDurationNs"])/1e3:12.1f} us {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:10.1f} us/call  {r["Name"][:110]}')
PY
rm -rf "$OUT/prof_rank"
cat "$OUT/ranker_kernel_stats.txt"
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
tail -1 "$OUT/bench_ranker.log" | cut -c1-600
