cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_onnx.py -m gpu > gpurun_out/t8.log 2>&1
rc=$?; tail -2 gpurun_out/t8.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/bench_onnx.py --batches 128 --precisions fp32 --images 2048 > gpurun_out/onnx_e2e2.log 2>&1
rc=$?; grep image_featurizer gpurun_out/onnx_e2e2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --rows 2000000 > gpurun_out/bench_2rank.log 2>&1
rc=$?; tail -1 gpurun_out/bench_2rank.log | cut -c1-900; exit $rc
