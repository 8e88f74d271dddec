#!/bin/bash
# Round-6 pass 8: full GPU suite + smoke on the current tree, then GBDT overlap A/B (SML_GBDT_OVERLAP 0 / 1 / 2),
# ranker IDX A/B, the pipelined ImageTransformer bench, and a kernel trace of the best headline form.
OUT=${1:-gpurun_out/r6p8}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 1000 python -u -m pytest -v --timeout 180 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
tail -1 "$OUT/smoke.log"
SML_GBDT_OVERLAP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py -k "batched or index_only" > "$OUT/pytest_ov1.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_ov1.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_ov1.log" | head -20; exit $rc; }
for v in 0 1 2 0 1 2; do
  SML_GBDT_OVERLAP=$v SML_GBDT_INIT_TIMING=1 timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_ov$v.log" 2>&1 || exit 1
  echo -n "ov=$v "; tail -1 "$OUT/bench_ov$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
done
for v in 0 1; do
  SML_GBDT_IDX=$v timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker_idx$v.log" 2>&1 || exit 1
  echo -n "ranker idx=$v "; tail -1 "$OUT/bench_ranker_idx$v.log" | cut -c1-240
done
timeout -k 10 400 python tools/bench_image.py --images 2048 > "$OUT/bench_image.log" 2>&1 || exit 1
grep -h img_per_s "$OUT/bench_image.log" | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
head -8 "$OUT/tree_breakdown.txt"
