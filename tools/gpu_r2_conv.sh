#!/bin/bash
# Conv tile sweep (SML_CONV_TILE) + ONNX GPU tests + ONNX DataFrame DP bench (pinned prefetch ring).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-conv}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_onnx.py tests/test_conv_mfma.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $OUT/pytest.log)"
[ $rc -ne 0 ] && exit $rc
for T in ${TILES:-default 64x64 128x64 64x128 128x128}; do
  if [ "$T" = default ]; then
    timeout -k 10 300 python tools/bench_conv.py > $OUT/conv_$T.log 2>&1 || exit $?
  elif [ "$T" = depth2 ]; then
    SML_CONV_DEPTH=2 timeout -k 10 300 python tools/bench_conv.py --no-ref > $OUT/conv_$T.log 2>&1 || exit $?
  elif [ "$T" = depth1 ]; then
    timeout -k 10 300 python tools/bench_conv.py --no-ref > $OUT/conv_$T.log 2>&1 || exit $?
  else
    SML_CONV_TILE=$T timeout -k 10 300 python tools/bench_conv.py --no-ref > $OUT/conv_$T.log 2>&1 || exit $?
  fi
  echo "$T: $(tail -1 $OUT/conv_$T.log)"
done
[ -n "$NO_E2E" ] && exit 0
timeout -k 10 600 python tools/bench_onnx.py > $OUT/bench_onnx.log 2>&1 || exit $?
grep '^{' $OUT/bench_onnx.log | cut -c1-200
timeout -k 10 600 python tools/bench_onnx_dp.py --images 4096 > $OUT/bench_onnx_dp.log 2>&1 || exit $?
grep '^{' $OUT/bench_onnx_dp.log | cut -c1-200
