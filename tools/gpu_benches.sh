#!/bin/bash
# Secondary benchmarks (BASELINE configs 3 and 5) on one MI355X, plus the VW GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_vw_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_vw.log 2>&1 && \
timeout -k 10 600 python tools/bench_ranker.py --steps 20 --warmup 3 > gpurun_out/bench_ranker.log 2>&1 && \
timeout -k 10 600 python tools/bench_vw.py --steps 3 --warmup 1 > gpurun_out/bench_vw.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
