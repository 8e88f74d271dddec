#!/bin/bash
# Round-5 pass 3: VALU-lean histogram / tree-walk kernels - GBDT + VW GPU tests, headline bench x2, fit trace.
OUT=${1:-gpurun_out/r5p3}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py tests/test_vw_gpu.py > "$OUT/pytest_gbdt_vw.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench2.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
