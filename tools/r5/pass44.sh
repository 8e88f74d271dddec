#!/bin/bash
# Round-5 pass 44: DRAM bytes of the partition / histogram kernels (FETCH_SIZE, WRITE_SIZE) against their useful
# bytes, 20-iteration fit; then the VW estimator's host profile.
OUT=${1:-gpurun_out/r5p44}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
GB="python3 bench.py --steps 1 --warmup 0 --iterations 20"
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "bpart|bhist|score_grad" \
    -d "$OUT/$name" -o "$name" "$@" -- $GB > "$OUT/$name.log" 2>&1
}
run fetch --pmc FETCH_SIZE && run write --pmc WRITE_SIZE
rc=$?
python3 tools/r5/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
find "$OUT" -name '*.csv' -size +2M -delete
cat "$OUT/summary.txt" | head -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_vw.py --steps 3 --warmup 1 --profile > "$OUT/bench_vw.log" 2> "$OUT/bench_vw_profile.txt" || exit 1
tail -1 "$OUT/bench_vw.log" | cut -c1-300
