#!/bin/bash
# Round-5 pass 9: the whole GPU suite in one process, smoke(), and the secondary benches (ResNet-50 session
# fp32 default = bf16x3 / fp16, ranker, VW estimator with fp32 sync sums and pooled buffers).
OUT=${1:-gpurun_out/r5p9}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest -v --timeout 180 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp32,fp16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rank" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_rank.log" 2>&1 || exit 1
