cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PAGEVEC_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --batch 1024 --recall 256 > gpurun_out/bench_2rank.log 2>&1
echo "2rank rc=$?"; tail -3 gpurun_out/bench_2rank.log
unset PAGEVEC_DIST_BACKEND
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench_1rank_torchrun.log 2>&1
echo "1rank rc=$?"; tail -1 gpurun_out/bench_1rank_torchrun.log
