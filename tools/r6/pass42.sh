#!/bin/bash
# Round-6 pass 42: secondary ONNX numbers on the final kernels - the ONNXModel DataFrame path (pass34's probe)
# and the ImageFeaturizer end-to-end legs over 2048 images.
OUT=${1:-gpurun_out/r6p42}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 python3 tools/r6/onnx_dp_cprofile.py > "$OUT/onnx_dp.log" 2>&1 || exit 1
grep -v "^ " "$OUT/onnx_dp.log" | grep -i "img" | head -5
timeout -k 10 400 python3 tools/bench_onnx.py --batches 256 --precisions fp32,fp16 --iters 20 --images 2048 > "$OUT/bench_onnx_2048.log" 2>&1 || exit 1
grep -E "resnet50_session|image_featurizer" "$OUT/bench_onnx_2048.log"
