#!/bin/bash
# Round-4 sixth GPU pass: VW -q regression probe with and without the constant-slot aggregation, VW GPU tests,
# stem-kernel tests and ResNet-50 session after the coalesced im2col. Usage: tools/gpu_r4_round6.sh OUTDIR
OUT=${1:-gpurun_out/r4r6}
mkdir -p "$OUT"
SML_VW_HOT_AGG=0 timeout -k 10 300 python tools/vw_quad_probe.py > "$OUT/vw_quad_probe_agg0.log" 2>&1 || exit 1
SML_VW_HOT_AGG=1 timeout -k 10 300 python tools/vw_quad_probe.py > "$OUT/vw_quad_probe_agg1.log" 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py -k "stem" > "$OUT/pytest_stem.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_vw_gpu.py > "$OUT/pytest_vw.log" 2>&1
