#!/bin/bash
# Round-5 pass 56: VW learn kernel time with and without the per-block global-state atomics (SML_VW_PROF_MODE=1,
# timing only), kernel API on a resident pass.
OUT=${1:-gpurun_out/r5p56}
mkdir -p "$OUT"
for m in 0 1 0 1; do
  SML_VW_PROF_MODE=$m timeout -k 10 300 python tools/bench_vw.py --api kernel --resident --steps 3 --warmup 1 > "$OUT/kernel_m$m.log" 2>&1 || exit 1
  echo "mode $m: $(tail -1 "$OUT/kernel_m$m.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_pass'])")"
done
