#!/bin/bash
# Round-4 twelfth GPU pass: row-staged stem kernel (the whole GPU suite first, then the stem probe against
# the gather / row-run forms, the ResNet-50 session at batch 128 / 256 and its kernel trace).
# Usage: tools/gpu_r4_round12.sh OUTDIR
OUT=${1:-gpurun_out/r4r12}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/stem_probe.py 128 20 > "$OUT/stem_probe.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 256 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1
