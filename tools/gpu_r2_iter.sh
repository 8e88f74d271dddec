#!/bin/bash
# One GBDT iteration on the GPU box: GBDT GPU tests, headline bench, and a kernel trace of a short bench.
# usage: TAG=name [TESTS=tests/test_gbdt_gpu.py] bash tools/gpu_r2_iter.sh
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-iter}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gbdt_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_$rep.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_$rep.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], 'ms/iter', d['config']['train_auc_all_rows'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o bench \
  -- python3 "$ROOT/bench.py" --steps 4 --warmup 1 > "$ROOT/$OUT/prof_stdout.log" 2>&1
echo "rocprof rc=$?"
