#!/bin/bash
# GBDT GPU tests, then an A/B of an env knob on the headline bench (same box, alternating runs).
# usage: KNOB=SML_FUSED_SPLIT A=0 B=1 bash tools/gpu_r2_ab.sh
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/ab_${KNOB}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gbdt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in $A $B; do
    env $KNOB=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_${v}_${rep}.log 2>&1 || exit $?
    echo "$KNOB=$v rep$rep $(python -c "import json,sys; d=json.loads(open('$OUT/bench_${v}_${rep}.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['train_auc_all_rows'])")"
  done
done
