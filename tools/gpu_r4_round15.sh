#!/bin/bash
# Round-4 fifteenth GPU pass: transpose-reduced lambdarank top sums (tests incl. the bitwise A/B, ranker fit
# with SML_RANK_TREDUCE=1 (default) and =0, kernel trace). Usage: tools/gpu_r4_round15.sh OUTDIR
OUT=${1:-gpurun_out/r4r15}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py -m gpu -k "rank or ndcg or metric" > "$OUT/pytest.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
SML_RANK_TREDUCE=0 timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker_tr0.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_ranker" -o ranker -- python3 tools/bench_ranker.py --steps 1 --warmup 1 > "$OUT/prof_ranker.log" 2>&1
