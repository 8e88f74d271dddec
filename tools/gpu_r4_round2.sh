#!/bin/bash
# Round-4 second GPU pass: GBDT batched growth (incremental replay) vs one-split growth and speculation widths,
# GBDT / VW / conv tests, ResNet-50 session with the stem kernel and LDS-DMA defaults, batched-fit profile.
# Usage: tools/gpu_r4_round2.sh OUTDIR
OUT=${1:-gpurun_out/r4r2}
mkdir -p "$OUT"
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
SML_GBDT_SPEC=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench_seq.log" 2>&1 || exit 1
for k in 2 4; do SML_GBDT_SPEC=$k timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench_spec$k.log" 2>&1 || exit 1; done
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py > "$OUT/pytest_gbdt.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py -k "stem or exact_integer or fp32_reference" > "$OUT/pytest_conv.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16,bf16,fp32 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
timeout -k 10 200 python tools/bench_conv.py --dtype fp16 --no-ref > "$OUT/conv_fp16_default.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_vw_gpu.py > "$OUT/pytest_vw.log" 2>&1
