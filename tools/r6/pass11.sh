#!/bin/bash
# Round-6 pass 11: expansion cursors on separate cache lines (partition claims stop serialising on one line);
# GBDT GPU tests, headline x2 with the partition tile A/B (SML_PART_ROWS 8 / 16) and a kernel breakdown.
OUT=${1:-gpurun_out/r6p11}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py -m gpu > "$OUT/pytest_gbdt.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gbdt.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gbdt.log" | head -20; exit $rc; }
for v in 8 16 8 16; do
  SML_PART_ROWS=$v timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_pr$v.log" 2>&1 || exit 1
  echo -n "part_rows=$v "; tail -1 "$OUT/bench_pr$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
head -8 "$OUT/tree_breakdown.txt"
sed -n '/batched growth/,$p' "$OUT/tree_breakdown.txt" | head -14
