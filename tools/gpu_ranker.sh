#!/bin/bash
# Ranker: GPU lambdarank tests, tools/bench_ranker.py, and a rocprofv3 kernel-stats run of it.
set -o pipefail
cd /root/repo; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gbdt_gpu.py -x -v --timeout 120 --timeout-method thread -k "rank or lambda" > gpurun_out/pytest_rank.log 2>&1 && \
timeout -k 10 300 python tools/bench_ranker.py > gpurun_out/bench_ranker.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/prof_rank -o rank -- python /root/repo/tools/bench_ranker.py --steps 10 > /root/repo/gpurun_out/prof_rank.log 2>&1
