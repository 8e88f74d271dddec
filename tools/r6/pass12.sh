#!/bin/bash
# Round-6 pass 12: pass 11 (cursor lines, part-rows A/B, breakdown) then pass 10 (fit overhead probe, 2/4-rank
# shared-device rehearsals with per-fit data-plane bytes) in one call.
ROOT=$(pwd)
bash tools/r6/pass11.sh gpurun_out/r6p12 || exit 1
cd "$ROOT" && bash tools/r6/pass10.sh gpurun_out/r6p12 || exit 1
