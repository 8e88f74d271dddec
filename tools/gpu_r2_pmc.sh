#!/bin/bash
# Round-2 PMC passes over the headline bench (one rocprofv3 run per pass, kernel trace + counters only).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out/pmc2"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, program args...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o "$name" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
GB="python3 $ROOT/bench.py --steps 2 --warmup 1"
run wave --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -- $GB && \
run lds --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- $GB && \
run l2 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -- $GB
rc=$?
python3 "$ROOT/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
exit $rc
