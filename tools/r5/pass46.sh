#!/bin/bash
# Round-5 pass 46: plan kernel for > 64 leaves without scratch (per-slot readlanes): GBDT GPU tests, the
# headline bench, and a 255-leaf fit (plan kernel time from the trace).
OUT=${1:-gpurun_out/r5p46}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || { grep -E "FAILED" "$OUT/pytest_gbdt.log" | head; exit 1; }
tail -1 "$OUT/pytest_gbdt.log"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof255" -o l255 -- python3 bench.py --steps 2 --warmup 1 --leaves 255 > "$OUT/bench_255.log" 2>&1 || exit 1
tail -1 "$OUT/bench_255.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('255 leaves', d['value'], d['ms_per_step'], d['config']['iteration_ms'])"
f=$(find "$OUT/prof255" -name '*kernel_stats.csv' -print -quit)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("bplan", "bhist", "bpart", "bfind", "breduce")):
        print(f'  {float(r["AverageNs"])/1e3:8.2f} us/call x {r["Calls"]}  {r["Name"][:60]}')
PY
rm -rf "$OUT/prof255"
