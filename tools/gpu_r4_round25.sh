#!/bin/bash
# Round-4 twenty-fifth GPU pass (no code change): 2-rank shared-device rehearsal of bench.py's data-parallel
# path on the final kernels, and a VW estimator kernel trace for the next round. Usage: tools/gpu_r4_round25.sh OUTDIR
OUT=${1:-gpurun_out/r4r25}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python bench.py --gpus 2 --allow-shared-device --rows 2000000 --steps 2 --warmup 1 > "$OUT/bench_2rank_shared.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_vw" -o vw -- python3 tools/bench_vw.py --steps 1 --warmup 1 > "$OUT/prof_vw.log" 2>&1
