#!/bin/bash
# Round-5 pass 27: bplan pop-loop shader clocks next to its wall time (SML_BPLAN_PROF).
OUT=${1:-gpurun_out/r5p27}
mkdir -p "$OUT"
SML_BPLAN_PROF=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 > "$OUT/bench_prof.log" 2> "$OUT/bplan_phases.txt" || exit 1
tail -3 "$OUT/bplan_phases.txt"
