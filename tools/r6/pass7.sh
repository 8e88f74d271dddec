#!/bin/bash
# Round-6 pass 7: two-stream overlap of partition / histograms (SML_GBDT_OVERLAP=k) - byte-identity tests
# under the knob, then bench A/B 0 / 1 / 2 and a kernel trace with overlap 1.
OUT=${1:-gpurun_out/r6p7}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
SML_GBDT_OVERLAP=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py -k "batched or index_only or trees_match or fans_out" > "$OUT/pytest_ov1.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_ov1.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_ov1.log" | head -20; exit $rc; }
SML_GBDT_OVERLAP=2 timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py -k "batched or index_only" > "$OUT/pytest_ov2.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_ov2.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_ov2.log" | head -20; exit $rc; }
for v in 0 1 2 0 1 2; do
  SML_GBDT_OVERLAP=$v timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_ov$v.log" 2>&1 || exit 1
  echo -n "ov=$v "; tail -1 "$OUT/bench_ov$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
done
SML_GBDT_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown_ov1.txt" 2>&1
cp "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" "$OUT/kernel_trace_ov1.csv"
rm -rf "$OUT/prof_fit"
head -8 "$OUT/tree_breakdown_ov1.txt"
