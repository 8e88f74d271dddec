#!/bin/bash
# Round-6 full check: the whole GPU suite in one process, smoke(), the headline bench.
OUT=${1:-gpurun_out/r6full}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench_default.log" 2>&1 || exit 1
tail -1 "$OUT/bench_default.log"
