#!/bin/bash
# Round-5 pass 57 (final, after the VW staging change): full GPU suite, smoke(), headline bench x2.
OUT=${1:-gpurun_out/r5p57}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 1000 python -u -m pytest -v --timeout 180 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && { grep -E "FAILED" "$OUT/pytest_gpu.log" | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
tail -1 "$OUT/smoke.log"
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
done
