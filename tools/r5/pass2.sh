#!/bin/bash
# Round-5 pass 2: PMC counters of the GBDT root pass and batched histogram / partition kernels (one rocprofv3
# run per counter set, kernel trace only), 20-iteration fits.
OUT=${1:-gpurun_out/r5p7}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
GB="python3 bench.py --steps 1 --warmup 0 --iterations 20"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "score_grad|bhist" \
    -d "$OUT/$name" -o "$name" "$@" -- $GB > "$OUT/$name.log" 2>&1
}
run valu --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR && \
run wait --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES && \
run lds --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT
rc=$?
python3 tools/r5/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
find "$OUT" -name '*.csv' -size +2M -delete
exit $rc
