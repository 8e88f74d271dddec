#!/bin/bash
# Round-4 seventh GPU pass: stem kernel (LDS pixel table) tests + session + trace; VW estimator / kernel benches;
# ranker fit after the lambdarank-init change. Usage: tools/gpu_r4_round7.sh OUTDIR
OUT=${1:-gpurun_out/r4r7}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py -k "stem" > "$OUT/pytest_stem.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --api kernel --steps 3 --warmup 1 > "$OUT/bench_vw_kernel.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_ranker" -o ranker -- python3 tools/bench_ranker.py --steps 1 --warmup 1 > "$OUT/prof_ranker.log" 2>&1
