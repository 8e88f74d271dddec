cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py tests/test_comm_gpu.py > gpurun_out/t1.log 2>&1
rc=$?
tail -3 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/b1.log 2>&1
rc=$?; tail -1 gpurun_out/b1.log; exit $rc
