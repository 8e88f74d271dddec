#!/bin/bash
# End-of-session HEAD check on one MI355X: every GPU test, smoke(), the headline bench, the ONNX / ImageFeaturizer
# benches and rocprofv3 kernel stats of the fit. Usage: tools/gpu_head_check.sh [out-subdir]
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
O="gpurun_out/${1:-head}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
tail -1 $O/tests.log; grep -E "^FAILED" $O/tests.log | head
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 400 python -u tools/bench_onnx.py --precisions fp32,fp32-bf16x3,fp16 --batches 128 --iters 10 --images 1024 --decoders native > $O/onnx.log 2>&1 || exit 1
grep -h '"images_per_s"' $O/onnx.log | cut -c1-200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o bench -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 > "$ROOT/$O/prof_stdout.log" 2>&1
