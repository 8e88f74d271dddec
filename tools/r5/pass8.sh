#!/bin/bash
# Round-5 pass 8: software-pipelined batched partition (A/B against the plain tile loop), GBDT GPU tests,
# then PMC counters of the root pass / histogram kernels on the VALU-lean code.
OUT=${1:-gpurun_out/r5p8}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || exit 1
for v in pipe nopipe pipe2 nopipe2; do
  case $v in nopipe*) export SML_PART_PIPE=0 ;; *) unset SML_PART_PIPE ;; esac
  timeout -k 10 300 python bench.py --steps 5 > "$OUT/bench_$v.log" 2>&1 || exit 1
done
unset SML_PART_PIPE
grep -o '"iteration_ms": [0-9.]*' "$OUT"/bench_*.log
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
bash tools/r5/pass2.sh "$OUT/pmc"
