#!/bin/bash
# Round-5 pass 6: device ImageTransformer (K19/K20) - GPU image tests, img/s bench, kernel trace; headline bench.
OUT=${1:-gpurun_out/r5p6}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_image.py -m gpu > "$OUT/pytest_image.log" 2>&1 || exit 1
timeout -k 10 300 python tools/bench_image.py --images 1024 --reps 3 > "$OUT/bench_image.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_image" -o img -- python3 tools/bench_image.py --images 512 --reps 1 > "$OUT/prof_image.log" 2>&1 || exit 1
find "$OUT/prof_image" -name '*kernel_stats.csv' -exec cp {} "$OUT/image_kernel_stats.csv" \;
rm -rf "$OUT/prof_image"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || exit 1
