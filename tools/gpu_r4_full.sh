#!/bin/bash
# Round-4 full GPU check (what the driver runs at round end): every GPU test in one process, smoke(), bench.
# Usage: tools/gpu_r4_full.sh OUTDIR
OUT=${1:-gpurun_out/r4full}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py > "$OUT/bench.log" 2>&1
