#!/bin/bash
# PMC passes over the ranker bench (lambdarank kernel): wave-level issue / wait counters and instruction mix.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out/${TAG:-rankpmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
D="python3 $ROOT/tools/bench_ranker.py --steps 2 --warmup 1"
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o "$name" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run wave --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -- $D || exit 1
run mix --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA -- $D || exit 1
python3 "$ROOT/tools/summarize_pmc.py" "$OUT" > "$OUT/summary.txt" 2>&1
grep -A 40 "lambdarank" "$OUT/summary.txt" | grep lambdarank | head -40
