#!/bin/bash
# Round-5 pass 13: lambdarank LPT order + LDS gain / top staging (tests, ranker kernel stats), VW shared pinned
# stager + device-packed model export (suite, bench with host profile), conv LDS-DMA issue schedules A/B.
OUT=${1:-gpurun_out/r5p13}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gbdt_gpu.py -k "rank" tests/test_vw_gpu.py tests/test_comm_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rank" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_rank.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 --profile > "$OUT/bench_vw_estimator.log" 2> "$OUT/bench_vw_profile.txt" || exit 1
tail -1 "$OUT/bench_vw_estimator.log"
for sc in 0 1 2; do
  SML_CONV_GLDS_SCHED=$sc timeout -k 10 300 python tools/bench_conv.py --no-ref > "$OUT/conv_sched$sc.log" 2>&1 || exit 1
done
grep TOTAL "$OUT"/conv_sched*.log
SML_CONV_GLDS_SCHED=1 timeout -k 10 300 $PYT tests/test_conv_mfma.py > "$OUT/pytest_conv_sched1.log" 2>&1 || { tail -30 "$OUT/pytest_conv_sched1.log"; exit 1; }
tail -1 "$OUT/pytest_conv_sched1.log"
