cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_vw_gpu.py tests/test_comm_gpu.py tests/test_gbdt_gpu.py -m gpu > gpurun_out/t4.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/t4.log | tail -80
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_vw.py --bits 26 --rows 1000000 --steps 3 > gpurun_out/vwb.log 2>&1
rc=$?
tail -3 gpurun_out/vwb.log
exit $rc
