#!/bin/bash
# MFMA conv kernel: numerics tests, then a micro-benchmark vs MIOpen (torch) per ResNet-50 layer shape.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests/test_conv_mfma.py -m gpu -x -q > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/pytest_conv.log
tail -30 gpurun_out/pytest_conv.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_conv.py > gpurun_out/bench_conv.log 2>&1 || exit $?
cat gpurun_out/bench_conv.log
