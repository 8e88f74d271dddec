#!/bin/bash
# List the PMC counters rocprofv3 exposes on this GPU (for choosing --pmc sets).
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$ROOT/gpurun_out/counters_avail.txt" 2>&1
echo "rc=$?"
grep -c . "$ROOT/gpurun_out/counters_avail.txt"
