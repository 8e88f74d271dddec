#!/bin/bash
# Round-6 pass 23: how much of the fused root pass (score_grad_hist_kernel) is the per-row tree walk -
# kernel stats with and without SML_PREP_NOWALK=1 (timing only).
OUT=${1:-gpurun_out/r6p23}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for v in 0 1; do
  SML_PREP_NOWALK=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_nowalk$v" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_nowalk$v.log" 2>&1 || exit 1
  f=$(find "$OUT/prof_nowalk$v" -name "*kernel_stats.csv" | head -1)
  echo "nowalk=$v"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'score_grad' in r['Name'] or 'bhist' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"
done
