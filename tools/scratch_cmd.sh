cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/s6
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_conv_mfma.py tests/test_onnx.py tests/test_gemm_gpu.py tests/test_dl_gpu.py tests/test_image.py > gpurun_out/s6/tests.log 2>&1
rc=$?; tail -3 gpurun_out/s6/tests.log | cut -c1-300; grep -E "FAILED|Error" gpurun_out/s6/tests.log | head -5; exit $rc
