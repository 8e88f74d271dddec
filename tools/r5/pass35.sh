#!/bin/bash
# Round-5 pass 35: rank-ordered replay frontier with children look-ahead (lane-coincidence fix): GBDT GPU tests, phase stamps, tree breakdown, bench.
OUT=${1:-gpurun_out/r5p35}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gbdt_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || { tail -40 "$OUT/pytest_gbdt.log"; exit 1; }
tail -1 "$OUT/pytest_gbdt.log"
SML_BPLAN_PROF=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > "$OUT/bench_prof.log" 2> "$OUT/bplan_phases.txt" || exit 1
tail -3 "$OUT/bplan_phases.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
head -8 "$OUT/tree_breakdown.txt"
grep bplan "$OUT/tree_breakdown.txt" | tail -1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
tail -1 "$OUT/bench.log" | cut -c1-400
