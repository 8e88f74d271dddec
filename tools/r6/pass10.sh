#!/bin/bash
# Round-6 pass 10: where a bench step's time goes outside the fit (probe), then the 2- and 4-rank shared-device
# rehearsals with per-fit data-plane bytes.
OUT=${1:-gpurun_out/r6p10}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 python tools/r6/fit_overhead_probe.py > "$OUT/fit_overhead_probe.log" 2>&1 || exit 1
grep step "$OUT/fit_overhead_probe.log"
for w in 2 4; do
  timeout -k 10 600 python bench.py --gpus $w --allow-shared-device --steps 2 --warmup 1 > "$OUT/bench_${w}rank_shared.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_${w}rank_shared.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print($w, d['value'], d['ms_per_step'], c['iteration_ms'], c['native_comm_ms'], c.get('native_comm_calls'), c.get('comm_bytes_bound'), c.get('comm_bytes_pushed'), c['histogram_allreduce'])"
done
