#!/bin/bash
# Round-4 eleventh GPU pass: row-run stem kernel (tests, probe vs the 2-byte gather form, session bench,
# texture-path counters) and 4-wave lambdarank blocks (tests, ranker fit A/B with SML_RANK_WAVES=1).
# Usage: tools/gpu_r4_round11.sh OUTDIR
OUT=${1:-gpurun_out/r4r11}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py tests/test_gbdt_gpu.py -m gpu -k "stem or resnet or rank or ndcg or metric" > "$OUT/pytest.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/stem_probe.py 128 20 > "$OUT/stem_probe.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
SML_RANK_WAVES=1 timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker_w1.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_onnx" -o onnx -- python3 tools/bench_onnx.py --batches 128 --precisions fp16 --images 0 > "$OUT/prof_onnx.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_ranker" -o ranker -- python3 tools/bench_ranker.py --steps 1 --warmup 1 > "$OUT/prof_ranker.log" 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE -d "$OUT/stem_ta" -o stem_ta -- python3 tools/stem_probe.py 128 3 > "$OUT/stem_ta.log" 2>&1
