#!/bin/bash
# Round-6 pass 17: ranker host phases (native parallel group-run scan, vectorised ideal DCG) - GBDT GPU tests,
# ranker bench x2, headline x1, ranker fault probe.
OUT=${1:-gpurun_out/r6p17b}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py -m gpu > "$OUT/pytest_gbdt.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gbdt.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gbdt.log" | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 400 python tools/bench_ranker.py > "$OUT/bench_ranker_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_ranker_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_fit'], d['iteration_ms'], d['fit_phases_ms'], d['group_prep_and_other_ms'])"
done
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_1.log" 2>&1 || exit 1
tail -1 "$OUT/bench_1.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
SML_GBDT_INIT_TIMING=1 timeout -k 10 400 python tools/r6/fit_fault_probe.py --ranker > "$OUT/faults_ranker.log" 2>&1 || exit 1
grep step "$OUT/faults_ranker.log" | tail -2; grep "objective init" "$OUT/faults_ranker.log" | tail -1
