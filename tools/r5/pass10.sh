#!/bin/bash
# Round-5 pass 10: the two pass-9 failures fixed (exact-mode fp32 conv test, VW sync sums scaled by 2^32),
# branch-free lambdarank pair terms (rcp instead of IEEE divides, scalar partner scores), and the 3-buffer
# LDS-DMA conv pipeline (SML_CONV_GLDS_NB=3) against the 2-buffer default per ResNet-50 layer.
OUT=${1:-gpurun_out/r5p10}
mkdir -p "$OUT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_comm_gpu.py tests/test_conv_mfma.py "tests/test_gbdt_gpu.py::test_gpu_lambdarank_gradients_match_host" "tests/test_gbdt_gpu.py::test_gpu_lambdarank_transpose_reduce_is_bitwise" > "$OUT/pytest_fix.log" 2>&1 || { tail -30 "$OUT/pytest_fix.log"; exit 1; }
tail -2 "$OUT/pytest_fix.log"
SML_CONV_GLDS_NB=3 timeout -k 10 400 $PYT tests/test_conv_mfma.py tests/test_onnx.py -m gpu > "$OUT/pytest_nb3.log" 2>&1 || { tail -30 "$OUT/pytest_nb3.log"; exit 1; }
tail -2 "$OUT/pytest_nb3.log"
timeout -k 10 300 python tools/bench_conv.py > "$OUT/conv_nb2.log" 2>&1 || exit 1
SML_CONV_GLDS_NB=3 timeout -k 10 300 python tools/bench_conv.py > "$OUT/conv_nb3.log" 2>&1 || exit 1
grep TOTAL "$OUT"/conv_nb*.log
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rank" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_rank.log" 2>&1 || exit 1
timeout -k 10 400 $PYT tests/test_vw_gpu.py > "$OUT/pytest_vw.log" 2>&1 || { tail -30 "$OUT/pytest_vw.log"; exit 1; }
tail -2 "$OUT/pytest_vw.log"
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
tail -1 "$OUT/bench_vw_estimator.log"
