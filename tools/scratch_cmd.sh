cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/s5
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/s5/tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/s5/bench.log 2>&1
rc=$?; tail -3 gpurun_out/s5/tests.log | cut -c1-300; tail -1 gpurun_out/s5/bench.log | cut -c1-700; exit $rc
