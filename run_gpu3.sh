cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/conv_micro.py --variants 0 --rounds 3 --bwd > gpurun_out/micro.log 2>&1; rc=$?; cat gpurun_out/micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b.log 2>&1; rc=$?; tail -1 gpurun_out/b.log
export PAGEVEC_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --batch 1024 --recall 256 > gpurun_out/bench_2rank.log 2>&1; rc=$?
echo "2rank rc=$rc"; tail -1 gpurun_out/bench_2rank.log | cut -c1-150
