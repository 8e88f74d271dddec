#!/bin/bash
# Round-4 ninth GPU pass: LDS-DMA conv with the fragment-time prologue (1x1 pre-activation layers):
# conv tests, ONNX session A/B (SML_CONV_GLDS_PRO=0 restores the register tiles there), kernel trace.
# Usage: tools/gpu_r4_round9.sh OUTDIR
OUT=${1:-gpurun_out/r4r9}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py -m gpu > "$OUT/pytest_conv_onnx.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
SML_CONV_GLDS_PRO=0 timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/bench_onnx_nopro.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/bench_onnx2.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1
