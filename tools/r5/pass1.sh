#!/bin/bash
# Round-5 pass 1: baseline on a fresh box - headline bench x2 and a kernel trace of the fit.
OUT=${1:-gpurun_out/r5p1}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench2.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
f=$(ls "$OUT"/prof_fit/*/fit_results.db "$OUT"/prof_fit/*/*kernel_trace.csv 2>/dev/null | head -n 1)
python tools/prof_tree_breakdown.py "$f" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
