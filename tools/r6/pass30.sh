#!/bin/bash
# Round-6 pass 30: VW touch map (sync epochs per 256-slot sub-block); the export skips never-written sub-blocks.
OUT=${1:-gpurun_out/r6p30}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_vw_gpu.py tests/test_vw.py -m gpu > "$OUT/pytest_vw.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_vw.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_vw.log" | head -20; exit $rc; }
timeout -k 10 300 python tools/r6/vw_contention_probe.py > "$OUT/contention.log" 2>&1 || exit 1
grep ids "$OUT/contention.log" | tail -2
for i in 1 2 3; do
  SML_VW_EXPORT_TIMING=1 timeout -k 10 400 python tools/bench_vw.py --steps 5 --warmup 1 > "$OUT/bench_vw_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_vw_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['phases_ms'], d['holdout_logloss'])"
done
grep "region scan" "$OUT/bench_vw_1.log" | tail -2
