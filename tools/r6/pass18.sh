#!/bin/bash
# Round-6 pass 18: VW staging - persistent copy team, binary-feature values as a device fill. VW GPU tests,
# VW bench x2 (+ fill off A/B), kernel trace of one VW bench.
OUT=${1:-gpurun_out/r6p18}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_vw_gpu.py -m gpu > "$OUT/pytest_vw.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_vw.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_vw.log" | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_vw_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['phases_ms'], d['holdout_logloss'])"
done
SML_VW_UNIT_FILL=0 timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_nofill.log" 2>&1 || exit 1
echo -n "no fill: "; tail -1 "$OUT/bench_vw_nofill.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['phases_ms'], d['holdout_logloss'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o vw -- python3 tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_prof.log" 2>&1 || exit 1
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$OUT/vw_kernel_stats.csv" && head -12 "$OUT/vw_kernel_stats.csv" | cut -c1-200
