#!/bin/bash
# Round-4 GPU check: GBDT bench (batched vs one-split growth), GBDT + VW GPU tests. Usage: tools/gpu_r4_check.sh OUTDIR
OUT=${1:-gpurun_out/r4}
mkdir -p "$OUT"
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
SML_GBDT_SPEC=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench_seq.log" 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_vw_gpu.py > "$OUT/pytest_vw.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py tests/test_comm_gpu.py > "$OUT/pytest_gbdt.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_onnx.py -k "gpu" > "$OUT/pytest_onnx.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/bench_transform.py > "$OUT/bench_transform.log" 2>&1
