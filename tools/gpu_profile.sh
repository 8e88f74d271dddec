#!/bin/bash
# rocprofv3 kernel-trace + stats of the flagship bench (no PMC counters here).
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/gpurun_out/prof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o bench \
  -- python3 "$ROOT/bench.py" --steps ${STEPS:-10} --warmup ${WARMUP:-2} ${BENCH_ARGS} > "$ROOT/gpurun_out/prof/bench_stdout.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$ROOT/gpurun_out/prof" -name "*stats*" | head
exit $rc
