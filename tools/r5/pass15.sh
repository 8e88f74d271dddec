#!/bin/bash
# Round-5 pass 15: lambdarank rank-loop partner source A/B (s_load / readlane / LDS), VW export phase timings.
OUT=${1:-gpurun_out/r5p15}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
for src in 0 1 2; do
  SML_RANK_SRC=$src timeout -k 10 300 $PYT "tests/test_gbdt_gpu.py::test_gpu_lambdarank_gradients_match_host" "tests/test_gbdt_gpu.py::test_gpu_lambdarank_ties_after_first_iteration" > "$OUT/pytest_src$src.log" 2>&1 || { tail -30 "$OUT/pytest_src$src.log"; exit 1; }
  SML_RANK_SRC=$src timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_src$src" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_src$src.log" 2>&1 || exit 1
  grep -i lambdarank_regs "$OUT/prof_src$src/rank_kernel_stats.csv" | awk -F, '{print "src'$src'", $(NF-5), $(NF-4)}'
done
SML_RANK_TREDUCE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_notr" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_notr.log" 2>&1 || exit 1
SML_VW_EXPORT_TIMING=1 timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2> "$OUT/vw_export_timing.txt" || exit 1
tail -1 "$OUT/bench_vw_estimator.log"
tail -12 "$OUT/vw_export_timing.txt"
