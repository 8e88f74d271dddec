#!/bin/bash
# GBDT GPU tests + headline bench (each GPU step under its own limit, chained with &&)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gbdt_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gbdt.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
