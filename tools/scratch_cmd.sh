cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/fpg
SML_HIST_FPG=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gbdt_gpu.py -k "trees_match or deterministic or quantisation" > gpurun_out/fpg/tests.log 2>&1 &&
for v in 32 16 32 16; do SML_HIST_FPG=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/fpg/bench_$v.log 2>&1 || exit 1; tail -1 gpurun_out/fpg/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($v, d['value'], d['config']['iteration_ms'], d['config']['fit_phases_ms'])"; done
rc=$?; tail -2 gpurun_out/fpg/tests.log; exit $rc
