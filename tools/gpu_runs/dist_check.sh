# Cross-GPU loss on one GPU: 2-rank gloo numerics test + a 2-rank gloo rehearsal of bench.py.
#   gpurun -- 'bash tools/gpu_runs/dist_check.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_dist.log
[ $rc -eq 0 ] || exit $rc
PAGEVEC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --batch 1024 --quality-steps 0 --recall 0 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "bench gloo2 rc=$rc"; tail -1 gpurun_out/bench_gloo2.log
