#!/bin/bash
# Round-4 third GPU pass: GBDT tests after the root-output fix, stem-kernel tests, speculation-width sweep,
# ResNet-50 session, then the estimator-level VW bench, comparators and the P2P probe.
# Usage: tools/gpu_r4_round3.sh OUTDIR
OUT=${1:-gpurun_out/r4r3}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py tests/test_comm_gpu.py > "$OUT/pytest_gbdt.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py -k "stem or split_k" tests/test_onnx.py > "$OUT/pytest_conv_onnx.log" 2>&1
rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench.log" 2>&1 || exit 1
for k in 3 5 6; do SML_GBDT_SPEC=$k timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench_spec$k.log" 2>&1 || exit 1; done
SML_GBDT_SPEC=0 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench_seq.log" 2>&1 || exit 1
SML_GBDT_LOOKAHEAD=2 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench_look2.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16,fp32 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx_dp.py --gpus 1 > "$OUT/bench_onnx_dp.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_transform.py > "$OUT/bench_transform.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29541 tools/p2p_check.py > "$OUT/p2p_check_2rank_1gpu.log" 2>&1
timeout -k 10 400 env OMP_NUM_THREADS=16 python tools/bench_comparators.py --which cpu,sklearn > "$OUT/comparators_11M_16threads.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --steps 2 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1
