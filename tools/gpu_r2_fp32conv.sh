#!/bin/bash
# fp32 MFMA conv: GPU tests (conv + ONNX), per-layer fp32 conv vs MIOpen, ResNet-50 session + DataFrame benches.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-fp32conv}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_conv_mfma.py tests/test_onnx.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest_conv.log)"
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/pytest_conv.log | head -20; exit $rc; }
timeout -k 10 300 python tools/bench_conv.py --dtype fp32 > $OUT/conv_fp32.log 2>&1 || exit $?
tail -3 $OUT/conv_fp32.log
for t in 64x64 64x128 128x64 128x128; do
  SML_CONV_TILE=$t timeout -k 10 300 python tools/bench_conv.py --dtype fp32 --no-ref > $OUT/sweep_fp32_$t.log 2>&1 || exit $?
  echo "$t $(tail -1 $OUT/sweep_fp32_$t.log)"
done
timeout -k 10 600 python tools/bench_onnx.py --batches 128 --precisions fp32,fp16 > $OUT/bench_onnx.log 2>&1 || exit $?
tail -4 $OUT/bench_onnx.log
timeout -k 10 600 python tools/bench_onnx_dp.py > $OUT/bench_onnx_dp.log 2>&1 || exit $?
tail -3 $OUT/bench_onnx_dp.log
