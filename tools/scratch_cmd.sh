cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gbdt_gpu.py -m gpu > gpurun_out/t10.log 2>&1
rc=$?; tail -3 gpurun_out/t10.log; [ $rc -ne 0 ] && exit $rc
for cfg in "SML_FUSE_HIST_FROM=0" "SML_FUSE_HIST_FROM=1" "SML_FUSE_HIST_FROM=1 SML_FUSED_ROWS=2" "SML_FUSE_HIST_FROM=1 SML_FUSED_ROWS=8" "SML_FUSE_HIST_FROM=4"; do
  env $cfg timeout -k 10 200 python bench.py --steps 4 --warmup 1 > gpurun_out/ab.log 2>&1 || exit $?
  tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$cfg', round(d['value']/1e6,2), c['iteration_ms'], c['fit_phases_ms']['training_iterations_ms'], c.get('holdout_auc_first_rows'))"
done
