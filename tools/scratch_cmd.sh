cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py -m gpu > gpurun_out/t6.log 2>&1
rc=$?; tail -3 gpurun_out/t6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_fused.log 2>&1 || exit $?
tail -1 gpurun_out/bench_fused.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('fused', d['value'], d['ms_per_step'], c['iteration_ms'], c['fit_phases_ms'])"
SML_FUSE_FIND=0 timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_unfused.log 2>&1 || exit $?
tail -1 gpurun_out/bench_unfused.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('unfused', d['value'], d['ms_per_step'], c['iteration_ms'], c['fit_phases_ms'])"
