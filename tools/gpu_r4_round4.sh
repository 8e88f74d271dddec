#!/bin/bash
# Round-4 fourth GPU pass: stem kernel (static-slot loads) tests + ResNet-50 session + kernel trace; VW estimator
# kernel trace (learn phase 94 ms vs the 28-ms kernel bench). Usage: tools/gpu_r4_round4.sh OUTDIR
OUT=${1:-gpurun_out/r4r4}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py -k "stem" tests/test_onnx.py > "$OUT/pytest_stem_onnx.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_onnx.py --batches 32,128 --precisions fp16,bf16 --images 512 > "$OUT/bench_onnx.log" 2>&1 || exit 1
SML_STEM_KERNEL=0 timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/bench_onnx_nostem.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_vw" -o vw -- python3 tools/bench_vw.py --steps 2 --warmup 1 > "$OUT/prof_vw.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --api kernel --steps 3 --warmup 1 > "$OUT/bench_vw_kernel.log" 2>&1
