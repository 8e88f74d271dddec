#!/bin/bash
# Round-6 pass 32: vectorised bins transpose - GBDT GPU tests, headline x2, kernel time of the transpose.
OUT=${1:-gpurun_out/r6p32}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py tests/test_comm_gpu.py -m gpu > "$OUT/pytest_gbdt.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gbdt.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gbdt.log" | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); grep -E "transpose|leaf_scatter|leaf_table|score_grad" "$f" | cut -d, -f1-5
