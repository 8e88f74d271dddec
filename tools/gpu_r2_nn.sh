#!/bin/bash
# ONNX / VW GPU tests (K13 hashing, K16 max pool) + ResNet-50 executor bench.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-nn}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_onnx.py tests/test_vw_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_onnx.py > $OUT/bench_onnx.log 2>&1 || exit $?
tail -4 $OUT/bench_onnx.log | cut -c1-300
