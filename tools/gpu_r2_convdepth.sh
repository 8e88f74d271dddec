#!/bin/bash
# A/B: fp32 conv one vs two register stages (SML_CONV_DEPTH), tests under depth 2, interleaved benches.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-convdepth}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
SML_CONV_DEPTH=2 timeout -k 10 300 python -u -m pytest tests/test_conv_mfma.py -m gpu -x -q -k fp32 --timeout 120 --timeout-method thread > $OUT/pytest_depth2.log 2>&1
rc=$?; echo "pytest depth2 rc=$rc $(tail -1 $OUT/pytest_depth2.log)"
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for d in 1 2; do
    SML_CONV_DEPTH=$d timeout -k 10 300 python tools/bench_conv.py --dtype fp32 --no-ref > $OUT/conv_d${d}_r$rep.log 2>&1 || exit $?
    echo "depth $d rep $rep $(tail -1 $OUT/conv_d${d}_r$rep.log)"
  done
done
for d in 1 2; do
  SML_CONV_DEPTH=$d timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp32 --images 0 > $OUT/session_d$d.log 2>&1 || exit $?
  echo "depth $d $(grep resnet50_session $OUT/session_d$d.log)"
done
