#!/bin/bash
# Round-6 pass 27: VW final export clears the table in place; the next fit reuses it without the memset.
OUT=${1:-gpurun_out/r6p27}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_vw_gpu.py -m gpu > "$OUT/pytest_vw.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_vw.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_vw.log" | head -20; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 400 python tools/bench_vw.py --steps 5 --warmup 1 > "$OUT/bench_vw_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_vw_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['phases_ms'], d['holdout_logloss'])"
done
SML_VW_CLEAN_TABLES=0 timeout -k 10 400 python tools/bench_vw.py --steps 5 --warmup 1 > "$OUT/bench_vw_noclean.log" 2>&1 || exit 1
echo -n "no clean: "; tail -1 "$OUT/bench_vw_noclean.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['phases_ms'], d['holdout_logloss'])"
