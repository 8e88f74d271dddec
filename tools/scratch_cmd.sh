cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_vw_gpu.py tests/test_comm_gpu.py -m gpu > gpurun_out/t9.log 2>&1
rc=$?; tail -2 gpurun_out/t9.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_vw.py --bits 30 --rows 2000000 --steps 3 > gpurun_out/vw_b30c.log 2>&1
rc=$?; tail -1 gpurun_out/vw_b30c.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_vw.py --bits 30 --rows 2000000 --steps 3 --resident > gpurun_out/vw_b30r.log 2>&1
rc=$?; tail -1 gpurun_out/vw_b30r.log; exit $rc
