#!/bin/bash
# Round-4 twenty-fourth GPU pass: gather stem kernel with its weight loads batched (conv + ONNX GPU tests,
# stem probe). Usage: tools/gpu_r4_round24.sh OUTDIR
OUT=${1:-gpurun_out/r4r24}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py -m gpu > "$OUT/pytest_conv.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/stem_probe.py 128 20 > "$OUT/stem_probe.log" 2>&1
