#!/bin/bash
# Round-5 pass 37: slab reduce + both children's searches in one launch (brfind_kernel, feature-major block
# slabs): GBDT GPU tests, tree breakdown, merged vs breduce + bfind.
OUT=${1:-gpurun_out/r5p37}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gbdt_gpu.py tests/test_comm_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || { grep -E "FAILED|Error|error" "$OUT/pytest_gbdt.log" | head -20; tail -5 "$OUT/pytest_gbdt.log"; exit 1; }
tail -1 "$OUT/pytest_gbdt.log"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
head -8 "$OUT/tree_breakdown.txt"
for v in merged split merged split; do
  if [ $v = split ]; then export SML_GBDT_MERGED_FIND=0; else unset SML_GBDT_MERGED_FIND; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$OUT/bench_$v.log" 2>&1 || exit 1
  echo "$v $(tail -1 "$OUT/bench_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['holdout_auc'])")"
done
