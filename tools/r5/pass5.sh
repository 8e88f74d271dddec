#!/bin/bash
# Round-5 pass 5: exact (int64, global-scale) data plane - GBDT GPU tests incl. 2-task shared-device bitwise
# equality and the world-1 RCCL path, headline bench, 2-rank shared-device bench rehearsal.
OUT=${1:-gpurun_out/r5p5}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py tests/test_comm_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 2 --allow-shared-device --steps 2 --warmup 1 > "$OUT/bench_2rank_shared.log" 2>&1 || exit 1
