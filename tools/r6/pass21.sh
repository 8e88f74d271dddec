#!/bin/bash
# Round-6 pass 21: PMC counters of the VW learn kernel (sgd_kernel) on tools/bench_vw.py (one counter pass per run).
OUT=${1:-gpurun_out/r6p21}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -oE "(TCC|TCP|TA|SQ)_[A-Z0-9_]*ATOM[A-Z0-9_]*" "$OUT/counters.txt" | sort -u > "$OUT/atomic_counters.txt" || true
p=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_FLAT" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum"; do
  p=$((p+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "sgd_kernel" --output-format csv -d "$OUT/pmc$p" -o vw -- python3 tools/bench_vw.py --steps 1 --warmup 1 > "$OUT/pmc$p.log" 2>&1 || echo "pass $p failed rc=$?"
done
ls -R "$OUT" | head -40
