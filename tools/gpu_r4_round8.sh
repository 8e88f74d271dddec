#!/bin/bash
# Round-4 eighth GPU pass: graph-capture test fix + the whole GPU suite; software-pipelined histogram loops
# (SML_GBDT_HIST_PIPE) A/B on the headline fit with a kernel trace of each. Usage: tools/gpu_r4_round8.sh OUTDIR
OUT=${1:-gpurun_out/r4r8}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > "$OUT/pytest_gpu.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench_base.log" 2>&1 || exit 1
SML_GBDT_HIST_PIPE=1 timeout -k 10 300 python bench.py > "$OUT/bench_pipe.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/bench_base2.log" 2>&1 || exit 1
SML_GBDT_HIST_PIPE=1 timeout -k 10 300 python bench.py > "$OUT/bench_pipe2.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_base" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_base.log" 2>&1 || exit 1
SML_GBDT_HIST_PIPE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_pipe" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_pipe.log" 2>&1
