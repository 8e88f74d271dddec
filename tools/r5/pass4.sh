#!/bin/bash
# Round-5 pass 4: branch-free tree-walk step; A/B of the histogram loop variants on the VALU-lean kernels.
OUT=${1:-gpurun_out/r5p4}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py > "$OUT/pytest_gbdt.log" 2>&1 || exit 1
for v in base pipe unroll4 base2; do
  case $v in
    pipe) export SML_GBDT_HIST_PIPE=1 ;;
    unroll4) unset SML_GBDT_HIST_PIPE; export SML_HIST_UNROLL=4 ;;
    *) unset SML_GBDT_HIST_PIPE SML_HIST_UNROLL ;;
  esac
  timeout -k 10 300 python bench.py --steps 5 > "$OUT/bench_$v.log" 2>&1 || exit 1
done
unset SML_GBDT_HIST_PIPE SML_HIST_UNROLL
grep -o '"iteration_ms": [0-9.]*' "$OUT"/bench_*.log
