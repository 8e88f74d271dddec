cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/cmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gbdt_gpu.py tests/test_comm_gpu.py > gpurun_out/cmp/tests.log 2>&1 &&
timeout -k 10 900 python -u tools/bench_comparators.py --which gpu,cpu,sklearn > gpurun_out/cmp/comparators.log 2>&1
rc=$?; tail -2 gpurun_out/cmp/tests.log; cut -c1-400 gpurun_out/cmp/comparators.log; exit $rc
