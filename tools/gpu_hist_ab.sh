#!/bin/bash
# A/B of histogram accumulation modes in one box (same device), then gpu tests.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for m in 0 1 2 1 0; do
  SML_HIST_MODE=$m timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ab_$m.log 2>&1 || exit $?
  echo "mode $m: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$m.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['train_auc_sample'])")"
done
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log
