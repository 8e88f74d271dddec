#!/bin/bash
# GBDT GPU loop: gbdt gpu tests, bench, rocprofv3 kernel stats.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_gbdt_gpu.py -m gpu -x -q > gpurun_out/pytest_gbdt.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/pytest_gbdt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || exit $?
cat gpurun_out/bench_full.log | tail -3
bash tools/gpu_profile.sh
