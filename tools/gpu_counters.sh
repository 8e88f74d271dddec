#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/runtime trace: each pass its own rocprofv3 run).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, program args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o "$name" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
GB="python3 $ROOT/bench.py --steps 3 --warmup 1"
# single-pass raw counters only (derived metrics such as FETCH_SIZE replay every dispatch many times)
run gbdt_lds --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES -- $GB && \
run gbdt_hbm --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -- $GB && \
run conv_mfma --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 "$ROOT/tools/bench_conv.py" --quick && \
run conv_hbm --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -- python3 "$ROOT/tools/bench_conv.py" --quick
rc=$?
python3 "$ROOT/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
exit $rc
