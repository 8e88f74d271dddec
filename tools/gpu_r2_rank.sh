#!/bin/bash
# GBDT GPU tests, headline bench, ranker bench + kernel trace.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-rank}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gbdt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log | cut -c1-250
timeout -k 10 600 python tools/bench_ranker.py --steps 20 --warmup 3 > $OUT/bench_ranker.log 2>&1 || exit $?
tail -1 $OUT/bench_ranker.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof_rank" -o rank \
  -- python3 "$ROOT/tools/bench_ranker.py" --steps 5 --warmup 1 > "$ROOT/$OUT/prof_rank.log" 2>&1
echo "rocprof rc=$?"
