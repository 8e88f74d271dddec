cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/vwflake
timeout -k 10 300 python -u tools/vw_flake_check.py 12 > gpurun_out/vwflake/alone.log 2>&1 || { tail -5 gpurun_out/vwflake/alone.log; exit 1; }
tail -1 gpurun_out/vwflake/alone.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_onnx_ops_ext.py tests/test_onnx.py tests/test_vw_gpu.py > gpurun_out/vwflake/seq.log 2>&1
rc=$?; tail -2 gpurun_out/vwflake/seq.log; exit $rc
