#!/bin/bash
# Round-5 pass 16: full GPU suite, smoke(), the headline bench (+ host profile of one fit), the ONNX fp32
# session kernel table.
OUT=${1:-gpurun_out/r5p16}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 1000 python -u -m pytest -v --timeout 180 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -4 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --profile > "$OUT/bench.log" 2> "$OUT/bench_profile.txt" || exit 1
tail -1 "$OUT/bench.log" | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_onnx32" -o onnx -- python3 tools/bench_onnx.py --batches 128 --precisions fp32 --images 0 > "$OUT/prof_onnx32.log" 2>&1 || exit 1
