#!/bin/bash
# A/B of GBDT launch shapes in one box (SML_PART_ROWS, SML_HIST_UNROLL); each run under its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
IFS=, read -ra CFGS <<< "${AB_CFGS:-16 4,8 4,4 4,16 8,8 8,16 2}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  SML_PART_ROWS=$1 SML_HIST_UNROLL=$2 SML_HIST_MIN_ROWS=${3:-2048} timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_p$1_h$2_m${3:-2048}.log 2>&1 || exit $?
  echo "part_rows=$1 hist_unroll=$2 hist_min_rows=${3:-2048} $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_p$1_h$2_m${3:-2048}.log)"
done
