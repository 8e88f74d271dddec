#!/bin/bash
# Round-4 twenty-third GPU pass (final state): the whole GPU suite in one process, smoke(), headline fit x2,
# ranker / VW estimator / ResNet-50 session benches, fit trace. Usage: tools/gpu_r4_round23.sh OUTDIR
OUT=${1:-gpurun_out/r4r23}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench2.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1
