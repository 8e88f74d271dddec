#!/bin/bash
# Round-6 pass 28: timeline of VW fits (kernels + memory copies) to find the engine's non-learning time.
OUT=${1:-gpurun_out/r6p28}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/prof" -o vw -- python3 tools/bench_vw.py --steps 2 --warmup 1 > "$OUT/bench_vw_prof.log" 2>&1 || exit 1
find "$OUT/prof" -name "*.csv" | head
