#!/bin/bash
# Round-6 pass 6: index-only partition - GBDT GPU tests, then bench A/B (SML_GBDT_IDX=0 / 1) and a kernel breakdown.
OUT=${1:-gpurun_out/r6p6}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py > "$OUT/pytest_gbdt_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gbdt_gpu.log"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gbdt_gpu.log" | head -20; exit $rc; }
for v in 0 1 0 1; do
  SML_GBDT_IDX=$v timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_idx$v.log" 2>&1 || exit 1
  echo -n "idx=$v "; tail -1 "$OUT/bench_idx$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
head -12 "$OUT/tree_breakdown.txt"
