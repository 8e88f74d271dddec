#!/bin/bash
# Round-6 pass 9: GBDT / VW / image GPU tests on the current tree, headline x2, a cProfile of one fit, the VW
# estimator bench (normalizer atomics skipped when they are no-ops), the image pipeline bench, and the 2-rank
# shared-device rehearsal with the data plane's byte counters.
OUT=${1:-gpurun_out/r6p9}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 800 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_gbdt_gpu.py tests/test_vw_gpu.py tests/test_image.py -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 1 > "$OUT/bench_$i.log" 2>&1 || exit 1
  tail -1 "$OUT/bench_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"
done
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --profile > "$OUT/bench_profile.log" 2> "$OUT/bench_profile.txt" || exit 1
head -45 "$OUT/bench_profile.txt" | tail -38 | cut -c1-150
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw.log" 2>&1 || exit 1
tail -1 "$OUT/bench_vw.log" | cut -c1-300
timeout -k 10 400 python tools/bench_image.py --images 2048 > "$OUT/bench_image.log" 2>&1 || exit 1
grep -h img_per_s "$OUT/bench_image.log" | head -6 | cut -c1-160
timeout -k 10 500 python bench.py --gpus 2 --allow-shared-device --steps 2 --warmup 1 > "$OUT/bench_2rank_shared.log" 2>&1 || exit 1
tail -1 "$OUT/bench_2rank_shared.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['iteration_ms'], c['native_comm_ms'], c.get('native_comm_calls'), c.get('comm_bytes_bound'), c.get('comm_bytes_pushed'), c['histogram_allreduce'])"
