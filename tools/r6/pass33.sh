#!/bin/bash
# Round-6 pass 33: the row -> leaf map in the plain score kernel (ranker, multiclass, regression).
OUT=${1:-gpurun_out/r6p33}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py tests/test_comm_gpu.py -m gpu > "$OUT/pytest_gbdt.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gbdt.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gbdt.log" | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 400 python tools/bench_ranker.py > "$OUT/bench_ranker_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_ranker_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['iteration_ms'], d['fit_phases_ms'])"
done
SML_GBDT_ROW_LEAF=0 timeout -k 10 400 python tools/bench_ranker.py > "$OUT/bench_ranker_walk.log" 2>&1 || exit 1
echo -n "walk: "; tail -1 "$OUT/bench_ranker_walk.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['iteration_ms'])"
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_1.log" 2>&1 || exit 1
tail -1 "$OUT/bench_1.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'])"
