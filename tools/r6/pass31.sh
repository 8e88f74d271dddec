#!/bin/bash
# Round-6 pass 31: VW export drain on the stager's copy team - VW export tests, VW bench x3.
OUT=${1:-gpurun_out/r6p31}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_vw_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest.log" | head -20; exit $rc; }
for i in 1 2 3; do
  SML_VW_EXPORT_TIMING=1 timeout -k 10 400 python tools/bench_vw.py --steps 5 --warmup 1 > "$OUT/bench_vw_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_vw_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['phases_ms'])"
done
grep "d2h" "$OUT/bench_vw_1.log" | tail -2
