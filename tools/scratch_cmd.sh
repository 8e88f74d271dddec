cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_onnx.py tests/test_gbdt_gpu.py -m gpu > gpurun_out/t7.log 2>&1
rc=$?; tail -3 gpurun_out/t7.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_onnx.py --batches 128 --precisions fp32,fp16 --images 2048 > gpurun_out/onnx_e2e.log 2>&1
rc=$?; grep image_featurizer gpurun_out/onnx_e2e.log; grep resnet50_session gpurun_out/onnx_e2e.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_r3c.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r3c.log | cut -c1-400; exit $rc
