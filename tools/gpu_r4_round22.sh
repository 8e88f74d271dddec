#!/bin/bash
# Round-4 twenty-second GPU pass: shorter replay argmax in the plan kernel (GBDT GPU tests,
# headline fit x2, kernel trace with the per-round breakdown). Usage: tools/gpu_r4_round22.sh OUTDIR
OUT=${1:-gpurun_out/r4r22}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py tests/test_lightgbm.py -m gpu > "$OUT/pytest_gbdt.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
[ $rc -eq 1 ] && exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench2.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1
