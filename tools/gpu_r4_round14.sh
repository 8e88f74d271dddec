#!/bin/bash
# Round-4 fourteenth GPU pass: lambdarank discount table from the host (tests, ranker fit, trace); stem
# affine loads hoisted (stem tests, probe, session at batch 256). Usage: tools/gpu_r4_round14.sh OUTDIR
OUT=${1:-gpurun_out/r4r14}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py tests/test_conv_mfma.py tests/test_onnx.py -m gpu -k "rank or ndcg or metric or stem or resnet" > "$OUT/pytest.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
timeout -k 10 120 python tools/stem_probe.py 128 20 > "$OUT/stem_probe.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 256 --precisions fp16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_ranker" -o ranker -- python3 tools/bench_ranker.py --steps 1 --warmup 1 > "$OUT/prof_ranker.log" 2>&1
