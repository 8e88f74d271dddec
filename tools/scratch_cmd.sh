cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_onnx.py tests/test_conv_mfma.py -m gpu > gpurun_out/t3.log 2>&1
rc=$?
tail -15 gpurun_out/t3.log
timeout -k 10 600 python tools/bench_onnx.py --batches 128 --precisions fp32,fp16 > gpurun_out/onnx1.log 2>&1
tail -8 gpurun_out/onnx1.log
exit $rc
