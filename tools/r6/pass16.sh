#!/bin/bash
# Round-6 pass 16: the secondary benches on the host-reuse tree - ranker fit (with the fit phases), VW fit,
# image pipeline, ONNX ResNet-50 fp32 / fp16, and the 2-rank shared-device rehearsal.
OUT=${1:-gpurun_out/r6p16}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 400 python tools/bench_ranker.py > "$OUT/bench_ranker.log" 2>&1 || exit 1
tail -1 "$OUT/bench_ranker.log" | cut -c1-600
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw.log" 2>&1 || exit 1
tail -1 "$OUT/bench_vw.log" | cut -c1-400
timeout -k 10 400 python tools/bench_image.py --images 2048 > "$OUT/bench_image.log" 2>&1 || exit 1
grep -h img_per_s "$OUT/bench_image.log" | head -6 | cut -c1-160
timeout -k 10 500 python tools/bench_onnx.py --batches 128,256 --precisions fp32,fp16 > "$OUT/bench_onnx.log" 2>&1 || exit 1
tail -6 "$OUT/bench_onnx.log" | cut -c1-300
timeout -k 10 500 python bench.py --gpus 2 --allow-shared-device --steps 2 --warmup 1 > "$OUT/bench_2rank_shared.log" 2>&1 || exit 1
tail -1 "$OUT/bench_2rank_shared.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['iteration_ms'], c['native_comm_ms'], c.get('native_comm_calls'), c.get('comm_bytes_bound'), c.get('comm_bytes_pushed'), c['fit_phases_ms'])"
