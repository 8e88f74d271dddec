#!/bin/bash
# Round-4 thirteenth GPU pass: row-staged stem with batched prologue loads and dword im2col (stem tests,
# probe, ResNet-50 session at batch 128 / 256, kernel trace). Usage: tools/gpu_r4_round13.sh OUTDIR
OUT=${1:-gpurun_out/r4r13}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py -m gpu -k "stem or resnet" > "$OUT/pytest_stem.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/stem_probe.py 128 20 > "$OUT/stem_probe.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 256 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1
