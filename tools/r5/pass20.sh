#!/bin/bash
# Round-5 pass 20: VW hogwild warm-up (launches of 1, 1, 2, 4, ... examples before the full batch): flake probe at
# batch 256 and 64, VW suite, VW bench.
OUT=${1:-gpurun_out/r5p20}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_vw_gpu.py tests/test_comm_gpu.py > "$OUT/pytest_vw.log" 2>&1 || { tail -40 "$OUT/pytest_vw.log"; exit 1; }
tail -1 "$OUT/pytest_vw.log"
timeout -k 10 300 python tools/r5/vw_flake_probe.py 8 256 > "$OUT/vw_flake_probe_b256.log" 2>&1 || exit 1
grep rep= "$OUT/vw_flake_probe_b256.log"
timeout -k 10 300 python tools/r5/vw_flake_probe.py 8 64 > "$OUT/vw_flake_probe_b64.log" 2>&1 || exit 1
grep rep= "$OUT/vw_flake_probe_b64.log"
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
tail -1 "$OUT/bench_vw_estimator.log"
SML_GBDT_INIT_TIMING=1 timeout -k 10 400 python bench.py --steps 2 --warmup 1 > "$OUT/bench_init_timing.log" 2> "$OUT/booster_init_timing.txt" || exit 1
tail -6 "$OUT/booster_init_timing.txt"
