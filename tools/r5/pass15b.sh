#!/bin/bash
# Round-5 pass 15b: pass 15 (lambdarank partner-source A/B, VW export timings) + pass 16 (full GPU suite,
# smoke, headline bench with a host profile, ONNX fp32 kernel table).
OUT=${1:-gpurun_out/r5p15}
bash tools/r5/pass15.sh "$OUT" || exit $?
bash tools/r5/pass16.sh "${OUT}_16"
