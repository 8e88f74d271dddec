#!/bin/bash
# Round-4 fifth GPU pass: VW device learner after the constant-slot aggregation and the parallel export
# (GPU tests incl. batch-1 parity, estimator and kernel benches, kernel trace), ranker fit after the
# lambdarank-init change. Usage: tools/gpu_r4_round5.sh OUTDIR
OUT=${1:-gpurun_out/r4r5}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_vw_gpu.py > "$OUT/pytest_vw.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --api kernel --steps 3 --warmup 1 > "$OUT/bench_vw_kernel.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_vw" -o vw -- python3 tools/bench_vw.py --steps 2 --warmup 1 > "$OUT/prof_vw.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_ranker" -o ranker -- python3 tools/bench_ranker.py --steps 1 --warmup 1 > "$OUT/prof_ranker.log" 2>&1
