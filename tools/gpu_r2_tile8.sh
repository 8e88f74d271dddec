#!/bin/bash
# f16/bf16 8-wave 128x128 tile rule: conv + ONNX GPU tests, per-layer (vs MIOpen), session and DataFrame benches.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-tile8}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_conv_mfma.py tests/test_onnx.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_conv.log)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_conv.py --dtype fp16 > $OUT/conv_fp16.log 2>&1 || exit $?
tail -1 $OUT/conv_fp16.log
timeout -k 10 600 python tools/bench_onnx.py --batches 128 --precisions fp32,fp16,bf16 > $OUT/bench_onnx.log 2>&1 || exit $?
grep '^{' $OUT/bench_onnx.log
timeout -k 10 600 python tools/bench_onnx_dp.py > $OUT/bench_onnx_dp.log 2>&1 || exit $?
grep '^{' $OUT/bench_onnx_dp.log
