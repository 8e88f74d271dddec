#!/bin/bash
# Round-2 baseline on a fresh box: GPU tests, headline bench, and a per-dispatch
# kernel trace of a short bench whose model is saved (leaf sizes per split).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
mkdir -p gpurun_out/r2base
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2base/pytest_gpu.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2base/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r2base/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/r2base/prof" -o bench \
  -- python3 "$ROOT/bench.py" --steps 4 --warmup 1 --save-model "$ROOT/gpurun_out/r2base/model.txt" \
  > "$ROOT/gpurun_out/r2base/prof_stdout.log" 2>&1
echo "rocprof rc=$?"
