#!/bin/bash
# lambdarank register path: GPU GBDT tests, ranker bench, ranker kernel stats.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-rank2}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gbdt_gpu.py tests/test_lightgbm.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gbdt.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gbdt.log)"
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/pytest_gbdt.log | head -20; exit $rc; }
timeout -k 10 600 python tools/bench_ranker.py --steps 20 --warmup 3 > $OUT/bench_ranker.log 2>&1 || exit $?
grep '^{' $OUT/bench_ranker.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof_rank" -o rank \
  -- python3 "$ROOT/tools/bench_ranker.py" --steps 5 --warmup 1 > "$ROOT/$OUT/prof_rank.log" 2>&1
echo "rocprof rc=$?"
grep -i lambdarank "$ROOT/$OUT/prof_rank/rank_kernel_stats.csv" | cut -c1-200
