cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/jpeg
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_image.py tests/test_onnx.py > gpurun_out/jpeg/tests.log 2>&1 &&
timeout -k 10 500 python -u tools/bench_onnx.py --precisions fp32 --batches 128 --iters 5 --images 2048 --decoders native,pil > gpurun_out/jpeg/bench.log 2>&1
rc=$?; tail -3 gpurun_out/jpeg/tests.log | cut -c1-300; cut -c1-260 gpurun_out/jpeg/bench.log | tail -8; exit $rc
