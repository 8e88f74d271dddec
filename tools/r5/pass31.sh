#!/bin/bash
# Round-5 pass 31: host phases of the fit (upload forms / threads, sample, bins), then the headline bench.
OUT=${1:-gpurun_out/r5p31}
mkdir -p "$OUT"
timeout -k 10 300 python tools/r5/fit_phase_probe.py > "$OUT/fit_phase_probe.log" 2>&1 || { tail -20 "$OUT/fit_phase_probe.log"; exit 1; }
cat "$OUT/fit_phase_probe.log"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['fit_phases_ms'])"
SML_UPLOAD_PIPE=0 timeout -k 10 300 python bench.py --steps 5 --warmup 1 > "$OUT/bench_pipe0.log" 2>&1 || exit 1
tail -1 "$OUT/bench_pipe0.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pipe0', d['value'], d['ms_per_step'], d['config']['fit_phases_ms'])"
