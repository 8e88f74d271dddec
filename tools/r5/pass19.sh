#!/bin/bash
# Round-5 pass 19: lambdarank launch split A/B (one launch / big + small NU<=2 launch / small launch in 4-wave
# blocks), rank tests, VW flake probe at batch 64 and the VW GPU suite.
OUT=${1:-gpurun_out/r5p19}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gbdt_gpu.py -k "rank" > "$OUT/pytest_rank.log" 2>&1 || { tail -40 "$OUT/pytest_rank.log"; exit 1; }
tail -1 "$OUT/pytest_rank.log"
timeout -k 10 400 $PYT tests/test_vw_gpu.py > "$OUT/pytest_vw.log" 2>&1 || { tail -40 "$OUT/pytest_vw.log"; exit 1; }
tail -1 "$OUT/pytest_vw.log"
SML_RANK_SMALL_WAVES=4 timeout -k 10 300 $PYT tests/test_gbdt_gpu.py -k "lambdarank" > "$OUT/pytest_rank_w4.log" 2>&1 || { tail -30 "$OUT/pytest_rank_w4.log"; exit 1; }
tail -1 "$OUT/pytest_rank_w4.log"
for cfg in "SML_RANK_SPLIT=0" "SML_RANK_SPLIT=1" "SML_RANK_SMALL_WAVES=4"; do
  ( export $cfg; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${cfg}" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_${cfg}.log" 2>&1 ) || exit 1
  echo "$cfg"; grep -i lambdarank_regs "$OUT/prof_${cfg}/rank_kernel_stats.csv" | awk -F, '{print $(NF-6), $(NF-5), $(NF-4)}'
done
timeout -k 10 300 python tools/r5/vw_flake_probe.py 6 64 > "$OUT/vw_flake_probe_b64.log" 2>&1 || exit 1
grep rep= "$OUT/vw_flake_probe_b64.log"
