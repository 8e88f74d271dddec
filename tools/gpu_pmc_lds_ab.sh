#!/bin/bash
# LDS counters (one PMC pass each) of the bench for the current GBDT extension and the saved baseline (ab_base/).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out/pmc_lds"
mkdir -p "$OUT"
so=$(ls "$ROOT"/synapseml_amd/_gbdt.cpython-*.so)
cp "$so" /tmp/new_gbdt.so
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$1" -o lds \
    --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES \
    -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 > "$OUT/$1.log" 2>&1 || exit $?
  echo "$1 rc=0"
}
run new
cp "$ROOT"/ab_base/_gbdt.cpython-*.so "$so"
run base
cp /tmp/new_gbdt.so "$so"
