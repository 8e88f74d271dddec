#!/bin/bash
# Round-6 pass 19: image batches' host side on a native thread team (gather into the pinned slot, per-row bytes
# split out of it) - image GPU tests, image bench, image cProfile.
OUT=${1:-gpurun_out/r6p19b}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_image.py tests/test_onnx.py -m gpu > "$OUT/pytest_image.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_image.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest_image.log" | head -20; exit $rc; }
timeout -k 10 400 python tools/bench_image.py --images 2048 > "$OUT/bench_image.log" 2>&1 || exit 1
grep -h img_per_s "$OUT/bench_image.log" | head -6 | cut -c1-160
timeout -k 10 400 python tools/r6/image_cprofile.py > "$OUT/image_cprofile.log" 2>&1 || exit 1
grep -A14 "== " "$OUT/image_cprofile.log" | cut -c1-150
