#!/bin/bash
# Round-4 seventeenth GPU pass (conv + GBDT): conv epilogue with its residual / affine loads batched ahead of
# the stores; branch-free batched loads in the GBDT partition / histogram / score kernels. Conv, ONNX and
# GBDT GPU tests; headline fit x2, ranker fit, ResNet-50 session (b128 / b256), per-layer conv sweep, fit
# trace. Usage: tools/gpu_r4_round17.sh OUTDIR
OUT=${1:-gpurun_out/r4r17}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py tests/test_gemm_gpu.py tests/test_dl_gpu.py tests/test_gbdt_gpu.py tests/test_lightgbm.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench2.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_default.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1
