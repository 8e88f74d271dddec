#!/bin/bash
# Last-split skip: GBDT GPU tests, then bench A/B (SML_SKIP_LAST_SPLIT=1 default vs 0), interleaved, + ranker.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-skiplast}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gbdt_gpu.py tests/test_lightgbm.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gbdt.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gbdt.log)"
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/pytest_gbdt.log | head -20; exit $rc; }
for rep in 1 2; do
  for v in 1 0; do
    SML_SKIP_LAST_SPLIT=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench_skip${v}_r$rep.log 2>&1 || exit $?
    echo "skip=$v rep $rep $(tail -1 $OUT/bench_skip${v}_r$rep.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
timeout -k 10 600 python tools/bench_ranker.py --steps 20 --warmup 3 > $OUT/bench_ranker.log 2>&1 || exit $?
grep '^{' $OUT/bench_ranker.log | grep -o '"ms_per_step": [0-9.]*\|"ndcg@10_holdout_slice": [0-9.]*'
