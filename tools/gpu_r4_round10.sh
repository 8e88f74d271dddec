#!/bin/bash
# Round-4 tenth GPU pass: stem kernel with the input BatchNormalization in its im2col (tests, probe, session
# bench), and the stem kernel's counters (what bounds it at ~313 us per batch of 128).
# Usage: tools/gpu_r4_round10.sh OUTDIR
OUT=${1:-gpurun_out/r4r10}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py -m gpu -k "stem or resnet or glds" > "$OUT/pytest_stem.log" 2>&1
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/stem_probe.py 128 20 > "$OUT/stem_probe.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_onnx.py --batches 128 --precisions fp16,bf16 --images 0 > "$OUT/bench_onnx.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || exit 1
have() { grep -q -w "$1" "$OUT/counters_list.txt"; }
pmc() {  # name, counters...
  local name=$1; shift
  local cs=""
  for c in "$@"; do have "$c" && cs="$cs $c"; done
  echo "$name:$cs" >> "$OUT/pmc_sets.txt"
  [ -z "$cs" ] && return 0
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $cs -d "$OUT/$name" -o "$name" -- python3 tools/stem_probe.py 128 3 > "$OUT/$name.log" 2>&1
}
pmc stem_sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD && \
pmc stem_sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC && \
pmc stem_ta TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
