#!/bin/bash
# Round-6 pass 40: env A/B of the conv forms on the ResNet-50 v2 session (fp16 / fp32, batch 256).
OUT=${1:-gpurun_out/r6p40}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for cfg in base SML_CONV_PERSIST=1 SML_CONV_GLDS_PRO=1 SML_CONV_SPLITK=auto; do
  if [ "$cfg" = base ]; then envs=""; else envs="$cfg"; fi
  env $envs timeout -k 10 300 python3 tools/bench_onnx.py --batches 256 --precisions fp16,fp32 --iters 30 --images 256 > "$OUT/bench_$cfg.log" 2>&1 || exit 1
  echo "$cfg"; grep resnet50_session "$OUT/bench_$cfg.log"
done
