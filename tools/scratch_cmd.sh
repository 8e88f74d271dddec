cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_vw_gpu.py tests/test_comm_gpu.py -m gpu > gpurun_out/vwt.log 2>&1
rc=$?
tail -30 gpurun_out/vwt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_vw.py --bits 26 --rows 1000000 --steps 3 > gpurun_out/vwb.log 2>&1
rc=$?
tail -3 gpurun_out/vwb.log
exit $rc
