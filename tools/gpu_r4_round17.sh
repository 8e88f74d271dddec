#!/bin/bash
# Round-4 seventeenth GPU pass: conv epilogue with its residual / affine loads batched ahead of the stores
# (all conv + ONNX GPU tests, per-layer sweep, ResNet-50 session at batch 128 / 256, kernel trace).
# Usage: tools/gpu_r4_round17.sh OUTDIR
OUT=${1:-gpurun_out/r4r17}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py tests/test_gemm_gpu.py tests/test_dl_gpu.py -m gpu > "$OUT/pytest_conv.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_default.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 256 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1
