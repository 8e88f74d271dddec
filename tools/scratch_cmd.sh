cd $GRAFT_REPO_ROOT
ROOT=$GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/s7
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/s7/tests.log 2>&1
tail -1 gpurun_out/s7/tests.log; grep -E "^FAILED" gpurun_out/s7/tests.log | head
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s7/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/s7/bench.log 2>&1 || exit 1
tail -1 gpurun_out/s7/bench.log | cut -c1-300
timeout -k 10 400 python -u tools/bench_onnx.py --precisions fp32,fp32-bf16x3,fp16 --batches 128 --iters 10 --images 1024 --decoders native > gpurun_out/s7/onnx.log 2>&1 || exit 1
grep -h '"images_per_s"' gpurun_out/s7/onnx.log | cut -c1-200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/s7/prof" -o bench -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 > "$ROOT/gpurun_out/s7/prof_stdout.log" 2>&1
