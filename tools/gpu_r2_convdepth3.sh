#!/bin/bash
# fp32 conv: epilogue pitch fix (auto depth) vs depth 3 (LDS fragment prefetch); tests under both, interleaved benches.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
OUT=gpurun_out/${TAG:-convdepth3}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for d in 0 3; do
  SML_CONV_DEPTH=$d timeout -k 10 300 python -u -m pytest tests/test_conv_mfma.py -m gpu -x -q -k fp32 --timeout 120 --timeout-method thread > $OUT/pytest_d$d.log 2>&1
  rc=$?; echo "pytest depth $d rc=$rc $(tail -1 $OUT/pytest_d$d.log)"
  [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
  for d in 0 3 1; do
    SML_CONV_DEPTH=$d timeout -k 10 300 python tools/bench_conv.py --dtype fp32 --no-ref > $OUT/conv_d${d}_r$rep.log 2>&1 || exit $?
    echo "depth $d rep $rep $(tail -1 $OUT/conv_d${d}_r$rep.log)"
  done
done
for d in 0 3; do
  SML_CONV_DEPTH=$d timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp32 --images 0 --iters 40 > $OUT/session_d$d.log 2>&1 || exit $?
  echo "depth $d $(grep resnet50_session $OUT/session_d$d.log)"
done
