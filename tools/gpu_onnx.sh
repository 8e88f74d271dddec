#!/bin/bash
# GPU check of the ONNX/image stack: gpu tests, throughput bench, kernel profile.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
mkdir -p gpurun_out/onnxprof
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_onnx.py ${ONNX_BENCH_ARGS} > gpurun_out/bench_onnx.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/onnxprof" -o onnx \
  -- python3 "$ROOT/tools/bench_onnx.py" --batches 128 --precisions fp16 --iters 10 --images 256 \
  > "$ROOT/gpurun_out/onnxprof/stdout.log" 2>&1
echo "rocprof rc=$?"
