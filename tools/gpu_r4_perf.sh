#!/bin/bash
# Round-4 performance pass: rocprofv3 kernel statistics of the headline fit (batched growth), estimator-level
# ranker / VW / transform benches, conv roofline table, P2P latency probe. Usage: tools/gpu_r4_perf.sh OUTDIR
OUT=${1:-gpurun_out/r4p}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fit" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit.log" 2>&1 || exit 1
SML_GBDT_SPEC=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_fit_seq" -o fit -- python3 bench.py --steps 2 --warmup 1 > "$OUT/prof_fit_seq.log" 2>&1 || exit 1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown_batched.txt" 2>&1
python3 tools/prof_tree_breakdown.py "$(find "$OUT/prof_fit_seq" -name '*kernel_trace.csv' -print -quit)" > "$OUT/tree_breakdown_sequential.txt" 2>&1
timeout -k 10 400 python tools/bench_ranker.py --steps 2 --warmup 1 > "$OUT/bench_ranker.log" 2>&1 || exit 1
timeout -k 10 400 python tools/bench_vw.py --steps 2 --warmup 1 > "$OUT/bench_vw_estimator.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_conv.py --dtype fp16 > "$OUT/conv_fp16_roofline.log" 2>&1 || exit 1
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29541 tools/p2p_check.py > "$OUT/p2p_check_2rank_1gpu.log" 2>&1 || true
timeout -k 10 400 env OMP_NUM_THREADS=16 python tools/bench_comparators.py --which cpu,sklearn > "$OUT/comparators_11M_16threads.log" 2>&1 || exit 1
for k in 4 12 16; do SML_GBDT_SPEC=$k timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench_spec$k.log" 2>&1 || exit 1; done
SML_GBDT_LOOKAHEAD=2 timeout -k 10 200 python bench.py --steps 3 --warmup 1 > "$OUT/bench_look2.log" 2>&1 || exit 1
