#!/bin/bash
# Round-6 pass 43: the multi-rank bench path on the rebuilt extensions (2 ranks sharing the box's one MI355X:
# a plumbing rehearsal of the driver's N-GPU run, not a scaling number).
OUT=${1:-gpurun_out/r6p43}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python bench.py --gpus 2 --allow-shared-device --steps 2 --warmup 1 > "$OUT/bench_2rank_shared.log" 2>&1 || exit 1
tail -1 "$OUT/bench_2rank_shared.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['iteration_ms'], c['native_comm_ms'], c.get('native_comm_calls'), c.get('comm_bytes_bound'), c.get('comm_bytes_pushed'), c['fit_phases_ms'])"
