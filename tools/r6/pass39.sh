#!/bin/bash
# Round-6 pass 39: 3x3 max pool with every tap load in flight: conv + ONNX GPU tests, then the fp32
# ResNet-50 session at batch 256 / 128 with kernel stats.
OUT=${1:-gpurun_out/r6p39}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_conv_mfma.py tests/test_onnx.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" "$OUT/pytest.log" | head -30; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fp32" -o onnx -- python3 tools/bench_onnx.py --batches 256 --precisions fp32 --iters 20 --images 256 > "$OUT/bench_fp32_prof.log" 2>&1 || exit 1
f=$(find "$OUT/prof_fp32" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_fp32.csv"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fp16" -o onnx -- python3 tools/bench_onnx.py --batches 256 --precisions fp16 --iters 20 --images 256 > "$OUT/bench_fp16_prof.log" 2>&1 || exit 1
f=$(find "$OUT/prof_fp16" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats_fp16.csv"
timeout -k 10 400 python3 tools/bench_onnx.py --batches 128,256 --precisions fp32,fp16 --iters 30 --images 256 > "$OUT/bench_onnx.log" 2>&1 || exit 1
grep resnet50_session "$OUT/bench_onnx.log"
