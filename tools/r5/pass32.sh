#!/bin/bash
# Round-5 pass 32: full GPU suite on the bplan rework, smoke(), the headline bench and its per-round breakdown.
OUT=${1:-gpurun_out/r5p32}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 1000 python -u -m pytest -v --timeout 180 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -4 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
tail -2 "$OUT/smoke.log"
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown.txt" 2>&1
rm -rf "$OUT/prof_fit"
head -8 "$OUT/tree_breakdown.txt"
