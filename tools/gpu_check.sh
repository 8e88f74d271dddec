#!/bin/bash
# First-pass GPU validation: tests, smoke, bench. Each GPU step has its own
# time limit; steps are chained with && so a failure stops the run.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
