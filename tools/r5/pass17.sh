#!/bin/bash
# Round-5 pass 17: CATS on the device (tests), VW suite + bench after the stats cleanup, headline bench with the
# parallel model text, ranker bench.
OUT=${1:-gpurun_out/r5p17}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_vw_gpu.py tests/test_lightgbm.py -m gpu > "$OUT/pytest_vw.log" 2>&1 || { tail -40 "$OUT/pytest_vw.log"; exit 1; }
tail -2 "$OUT/pytest_vw.log"
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
tail -1 "$OUT/bench_vw_estimator.log"
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
tail -1 "$OUT/bench.log" | cut -c1-300
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
tail -1 "$OUT/bench_ranker.log" | cut -c1-300
