#!/bin/bash
# Round-6 pass 14: the fitted model's training state released on a background thread (joined by the next
# fit's booster init) - GPU suite for the GBDT engine, headline x3 and the overhead probe.
OUT=${1:-gpurun_out/r6p14}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py tests/test_comm_gpu.py -m gpu > "$OUT/pytest_gbdt.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gbdt.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gbdt.log" | head -20; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
done
SML_GBDT_ASYNC_RELEASE=0 timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_sync_release.log" 2>&1 || exit 1
echo -n "sync release: "; tail -1 "$OUT/bench_sync_release.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
timeout -k 10 400 python tools/r6/fit_overhead_probe.py > "$OUT/fit_overhead_probe.log" 2>&1 || exit 1
grep step "$OUT/fit_overhead_probe.log"
