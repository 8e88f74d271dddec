#!/bin/bash
# Round-5 pass 14: lambdarank partner scores from LDS (ranker kernel stats), VW constructor without a wait +
# one-scan export (VW suite, bench), conv NB rule (blocks <= CUs) per-layer sweep, ONNX fp16/fp32.
OUT=${1:-gpurun_out/r5p14}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_vw_gpu.py tests/test_comm_gpu.py "tests/test_gbdt_gpu.py::test_gpu_lambdarank_gradients_match_host" "tests/test_gbdt_gpu.py::test_gpu_lambdarank_monotone_gain_form_is_bitwise" "tests/test_gbdt_gpu.py::test_gpu_lambdarank_ties_after_first_iteration" "tests/test_gbdt_gpu.py::test_gpu_lambdarank_transpose_reduce_is_bitwise" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rank" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_rank.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
tail -1 "$OUT/bench_ranker.log" | cut -c1-300
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
tail -1 "$OUT/bench_vw_estimator.log"
timeout -k 10 300 python tools/bench_conv.py --no-ref > "$OUT/conv_auto.log" 2>&1 || exit 1
SML_CONV_GLDS_NB=2 timeout -k 10 300 python tools/bench_conv.py --no-ref > "$OUT/conv_nb2.log" 2>&1 || exit 1
grep TOTAL "$OUT"/conv_*.log
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp32,fp16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
grep -h images_per_s "$OUT/bench_onnx.log"
