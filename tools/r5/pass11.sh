#!/bin/bash
# Round-5 pass 11: VW b30-scoring bisect (fused stage+learn on / off after the CB tests), the VW suite,
# the VW estimator bench + kernel trace, lambdarank PMC counters, ONNX ResNet-50 with the auto 3-buffer conv
# rule, smoke().
OUT=${1:-gpurun_out/r5p11}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
SML_VW_STAGE_LEARN=1 timeout -k 10 300 $PYT tests/test_vw_gpu.py -k "contextual or b30" > "$OUT/bisect_fused.log" 2>&1
echo "fused rc=$?"
SML_VW_STAGE_LEARN=0 timeout -k 10 300 $PYT tests/test_vw_gpu.py -k "contextual or b30" > "$OUT/bisect_plain.log" 2>&1
echo "plain rc=$?"
timeout -k 10 300 $PYT tests/test_vw_gpu.py -k "b30" > "$OUT/b30_alone.log" 2>&1
echo "alone rc=$?"
timeout -k 10 400 $PYT tests/test_vw_gpu.py tests/test_comm_gpu.py > "$OUT/pytest_vw.log" 2>&1
echo "vw suite rc=$?"; tail -3 "$OUT/pytest_vw.log"
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
tail -1 "$OUT/bench_vw_estimator.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_vw" -o vw -- python3 tools/bench_vw.py --steps 1 --warmup 1 > "$OUT/prof_vw.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128,256 --precisions fp32,fp16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
RK="python3 tools/bench_ranker.py --steps 1 --warmup 0"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "lambdarank" -d "$OUT/rank_valu" -o valu \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR -- $RK > "$OUT/rank_valu.log" 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "lambdarank" -d "$OUT/rank_wait" -o wait \
  --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES -- $RK > "$OUT/rank_wait.log" 2>&1 || exit 1
python3 tools/r5/pmc_summary.py "$OUT" > "$OUT/pmc_summary.txt" 2>&1
find "$OUT" -name '*.csv' -size +2M -delete
