#!/bin/bash
# rocprofv3 kernel-trace + stats of an arbitrary python benchmark: NAME=<tag> bash tools/gpu_prof_cmd.sh <script> [args...]
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME=${NAME:-prof}
OUT="$ROOT/gpurun_out/prof_$NAME"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
  -- python3 "$ROOT/$1" "${@:2}" > "$OUT/stdout.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
exit $rc
