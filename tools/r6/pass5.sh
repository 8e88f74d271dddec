#!/bin/bash
# Round-6 pass 5: DRAM bytes (FETCH_SIZE / WRITE_SIZE) and wave / instruction counters of the leaf-id partition
# and its histogram against the moving partition (SML_GBDT_LID=0 / 1), 20-iteration fits.
OUT=${1:-gpurun_out/r6p5}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
GB="python3 bench.py --steps 1 --warmup 0 --iterations 20"
run() {
  local name=$1 lid=$2; shift 2
  SML_GBDT_LID=$lid timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "bpart|bhist" \
    -d "$OUT/$name" -o "$name" "$@" -- $GB > "$OUT/$name.log" 2>&1
}
for lid in 0 1; do
  run fetch$lid $lid --pmc FETCH_SIZE && run write$lid $lid --pmc WRITE_SIZE && \
  run sq$lid $lid --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES || exit 1
done
python3 tools/r5/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
find "$OUT" -name '*.csv' -size +2M -delete
cat "$OUT/summary.txt" | head -120
