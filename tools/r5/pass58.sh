#!/bin/bash
# Round-5 pass 58: the logistic clamp as two scalars (no per-example bound arrays); as pass 55:
# the pinned stager: VW GPU tests, estimator bench x2, fit timeline.
OUT=${1:-gpurun_out/r5p58}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_vw_gpu.py > "$OUT/pytest_vw.log" 2>&1 || { grep -E "FAILED|Error" "$OUT/pytest_vw.log" | head; tail -3 "$OUT/pytest_vw.log"; exit 1; }
tail -1 "$OUT/pytest_vw.log"
for i in 1 2; do
  timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_vw_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['phases_ms'], d['holdout_logloss'])"
done
bash tools/r5/pass54.sh "$OUT/timeline" > /dev/null 2>&1 && sed -n '1,10p' "$OUT/timeline/timeline.txt"
