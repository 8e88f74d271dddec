#!/bin/bash
# GBDT GPU tests under each value of an env knob, then alternating headline benches (same box).
# usage: KNOB=SML_HIST_SHAPE VALS="0 1 2" bash tools/gpu_r2_ab3.sh
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/ab_${KNOB}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for v in $VALS; do
  env $KNOB=$v timeout -k 10 600 python -u -m pytest tests/test_gbdt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$KNOB=$v pytest rc=$rc $(tail -1 $OUT/pytest_$v.log)"
  [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
  for v in $VALS; do
    env $KNOB=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_${v}_${rep}.log 2>&1 || exit $?
    echo "$KNOB=$v rep$rep $(python -c "import json,sys; d=json.loads(open('$OUT/bench_${v}_${rep}.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['train_auc_all_rows'])")"
  done
done
