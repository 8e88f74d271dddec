cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/split3
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_mfma.py tests/test_onnx.py -m gpu > gpurun_out/split3/tests.log 2>&1 || { tail -40 gpurun_out/split3/tests.log; exit 1; }
tail -1 gpurun_out/split3/tests.log
timeout -k 10 400 python -u tools/bench_onnx.py --precisions fp32-exact,fp32-bf16x6,fp32-bf16x3 --batches 128 --iters 10 --images 256 --decoders native > gpurun_out/split3/onnx.log 2>&1 || exit 1
grep resnet50_session gpurun_out/split3/onnx.log | cut -c1-200
