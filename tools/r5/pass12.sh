#!/bin/bash
# Round-5 pass 12: lambdarank strict ranks + monotone-gain pair terms (tests, ranker bench, kernel stats),
# ONNX ResNet-50 fp16 with the 2-buffer conv forced vs the auto 3-buffer rule, and TA / SQ counters of the
# 3x3 conv layers.
OUT=${1:-gpurun_out/r5p12}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gbdt_gpu.py -k "rank" > "$OUT/pytest_rank.log" 2>&1 || { tail -40 "$OUT/pytest_rank.log"; exit 1; }
tail -2 "$OUT/pytest_rank.log"
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
tail -1 "$OUT/bench_ranker.log" | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rank" -o rank -- python3 tools/bench_ranker.py --steps 1 --warmup 0 > "$OUT/prof_rank.log" 2>&1 || exit 1
grep -i lambdarank "$OUT/prof_rank/rank_kernel_stats.csv" | cut -c1-160
SML_CONV_GLDS_NB=2 timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16 --images 0 > "$OUT/bench_onnx_nb2.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp16 --images 0 > "$OUT/bench_onnx_auto.log" 2>&1 || exit 1
grep -h images_per_s "$OUT"/bench_onnx_*.log
CV="python3 tools/bench_conv.py --only 1,4,8,11 --no-ref --quick"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "conv_glds" \
    -d "$OUT/$name" -o "$name" "$@" -- $CV > "$OUT/$name.log" 2>&1
}
run ta --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE && \
run sq1 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD && \
run sq2 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC
rc=$?
python3 tools/r5/pmc_summary.py "$OUT" conv_glds > "$OUT/conv_pmc_summary.txt" 2>&1
find "$OUT" -name '*.csv' -size +2M -delete
exit $rc
