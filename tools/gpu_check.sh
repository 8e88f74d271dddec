#!/bin/bash
# First-pass GPU validation: tests, small bench, full bench. Each GPU step has
# its own time limit; steps are chained with && so a failure stops the run.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" | tee -a gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --rows 1000000 --steps 10 --warmup 2 > gpurun_out/bench_small.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1
echo "bench rc=$?"
