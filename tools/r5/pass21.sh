#!/bin/bash
# Round-5 pass 21: headline bench with the integer-count start score (+ booster init phases), GBDT GPU tests.
OUT=${1:-gpurun_out/r5p21}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gbdt_gpu.py tests/test_comm_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || { tail -40 "$OUT/pytest_gbdt.log"; exit 1; }
tail -1 "$OUT/pytest_gbdt.log"
SML_GBDT_INIT_TIMING=1 timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench.log" 2> "$OUT/booster_init_timing.txt" || exit 1
tail -1 "$OUT/bench.log" | cut -c1-300
tail -6 "$OUT/booster_init_timing.txt"
