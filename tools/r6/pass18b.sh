OUT=gpurun_out/r6p18b; mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o vw -- python3 tools/bench_vw.py --steps 3 --warmup 1 > "$OUT/bench_vw_prof.log" 2>&1 || exit 1
find $OUT/prof -name "*.csv" | head
