#!/bin/bash
# PMC passes over single conv shapes (one rocprofv3 run per pass; counters only with kernel trace).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out/${TAG:-convpmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o "$name" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
# PMC_SHAPES: comma-separated C_H_Cout_k_stride list; MOPS: the MFMA op counter (..._F32 for fp32 runs)
for N in $(echo ${PMC_SHAPES:-1024_14_256_1_1,128_28_128_3_1} | tr ',' ' '); do
  SH=$(echo $N | tr '_' ' ')
  D="python3 $ROOT/tools/conv_pmc_driver.py $SH 20"
  run ${N}_wave --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -- $D || exit 1
  run ${N}_mfma --pmc ${MOPS:-SQ_INSTS_VALU_MFMA_MOPS_F16} SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE -- $D || exit 1
  run ${N}_l2 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -- $D || exit 1
done
python3 "$ROOT/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt" | head -80
