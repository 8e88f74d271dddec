#!/bin/bash
# Round-6 pass 20: adaptive round width (bplan keeps speculating while the round's expansions are small).
# Byte-identity tests, then the headline at several SML_GBDT_WIDE / SML_GBDT_SPEC_MAX settings.
OUT=${1:-gpurun_out/r6p20}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py -m gpu -k "adaptive_round_width or batched_growth_equals or index_only" > "$OUT/pytest_wide.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_wide.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_wide.log" | head -20; exit $rc; }
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_$label.log" 2>&1 || exit 1
  echo -n "$label: "; tail -1 "$OUT/bench_$label.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'])"
}
run base SML_GBDT_WIDE=0
run w8_m8 SML_GBDT_WIDE=8 SML_GBDT_SPEC_MAX=8
run w16_m8 SML_GBDT_WIDE=16 SML_GBDT_SPEC_MAX=8
run w32_m8 SML_GBDT_WIDE=32 SML_GBDT_SPEC_MAX=8
run w16_m12 SML_GBDT_WIDE=16 SML_GBDT_SPEC_MAX=12
run w64_m12 SML_GBDT_WIDE=64 SML_GBDT_SPEC_MAX=12
run base2 SML_GBDT_WIDE=0
