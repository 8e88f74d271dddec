#!/bin/bash
# fp32 conv depth rule (auto) vs forced 1 / 2: conv tests under auto and forced 2, per-layer and session benches.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-convdepth2}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_conv_mfma.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_auto.log 2>&1
rc=$?; echo "pytest auto rc=$rc $(tail -1 $OUT/pytest_auto.log)"
[ $rc -ne 0 ] && exit $rc
for d in 0 1 2; do
  SML_CONV_DEPTH=$d timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp32 --images 0 --iters 40 > $OUT/session_d$d.log 2>&1 || exit $?
  echo "depth $d $(grep resnet50_session $OUT/session_d$d.log)"
done
SML_CONV_DEPTH=0 timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp32 --images 0 --iters 40 > $OUT/session_d0b.log 2>&1 || exit $?
echo "depth 0 again $(grep resnet50_session $OUT/session_d0b.log)"
