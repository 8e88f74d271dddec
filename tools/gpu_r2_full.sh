#!/bin/bash
# Round-2 broad check: every GPU test, headline bench, ranker + VW + ONNX DP benches, ranker kernel trace.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_gpu.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 600 python tools/bench_ranker.py --steps 20 --warmup 3 > $OUT/bench_ranker.log 2>&1 || exit $?
tail -2 $OUT/bench_ranker.log | cut -c1-400
timeout -k 10 600 python tools/bench_vw.py --steps 3 --warmup 1 > $OUT/bench_vw.log 2>&1 || exit $?
tail -2 $OUT/bench_vw.log | cut -c1-400
timeout -k 10 600 python tools/bench_onnx_dp.py > $OUT/bench_onnx_dp.log 2>&1 || exit $?
tail -2 $OUT/bench_onnx_dp.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof_rank" -o rank \
  -- python3 "$ROOT/tools/bench_ranker.py" --steps 5 --warmup 1 > "$ROOT/$OUT/prof_rank.log" 2>&1
echo "rocprof rc=$?"
cd "$ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
echo "smoke rc=$? $(tail -1 $OUT/smoke.log)"
