#!/bin/bash
# Round-4 conv pass: MFMA conv tests (new tiles, LDS-DMA form, split-K), per-layer fp16 roofline sweeps per tile
# form, ResNet-50 session A/B (split-K, LDS-DMA). Usage: tools/gpu_r4_conv.sh OUTDIR
OUT=${1:-gpurun_out/r4conv}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_gemm_gpu.py > "$OUT/pytest_conv.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_default.log" 2>&1 || exit 1
SML_CONV_TILE=256x64 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_256x64.log" 2>&1 || exit 1
SML_CONV_TILE=128x164 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_128x64w2.log" 2>&1 || exit 1
SML_CONV_TILE=128x777 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_glds128.log" 2>&1 || exit 1
SML_CONV_TILE=64x777 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_glds64.log" 2>&1 || exit 1
SML_CONV_TILE=256x777 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_glds256x64.log" 2>&1 || exit 1
SML_CONV_TILE=128x932 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_m32_128.log" 2>&1 || exit 1
SML_CONV_TILE=256x932 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_m32_256x128.log" 2>&1 || exit 1
SML_CONV_TILE=64x932 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_m32_64.log" 2>&1 || exit 1
SML_CONV_PERSIST=1 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_persist.log" 2>&1 || exit 1
SML_CONV_SPLITK=0 timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_nosplitk.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16,fp32 > "$OUT/bench_onnx.log" 2>&1 || exit 1
SML_CONV_SPLITK=0 timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16 > "$OUT/bench_onnx_nosplitk.log" 2>&1 || exit 1
SML_CONV_PERSIST=1 timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16 > "$OUT/bench_onnx_persist.log" 2>&1 || exit 1
SML_CONV_GLDS=1 timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16 > "$OUT/bench_onnx_glds.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1 || exit 1
