#!/bin/bash
# Round-4 twenty-first GPU pass: single-buffer LDS-DMA conv for one-K-tile layers (conv + ONNX tests, session
# A/B with SML_CONV_GLDS_SINGLE=0, per-layer sweep). Usage: tools/gpu_r4_round21.sh OUTDIR
OUT=${1:-gpurun_out/r4r21}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py -m gpu > "$OUT/pytest_conv.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
SML_CONV_GLDS_SINGLE=0 timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16 --images 0 > "$OUT/bench_onnx_double.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16 --images 0 > "$OUT/bench_onnx2.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_default.log" 2>&1 || exit 1
SML_CONV_GLDS_SINGLE=0 timeout -k 10 300 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_double.log" 2>&1
