cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 0 --recall 0 --eager-compare 0 > gpurun_out/bench_eager.log 2>&1
rc=$?; echo "bench eager rc=$rc"; tail -1 gpurun_out/bench_eager.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ib_micro.py --M 16384,65536,131072 > gpurun_out/ib_micro.log 2>&1
rc=$?; echo "ib rc=$rc"; cat gpurun_out/ib_micro.log | tail -5
[ $rc -eq 0 ] || exit $rc
PAGEVEC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --recall 0 > gpurun_out/bench_gloo2.log 2>&1
rc=$?; echo "gloo2 rc=$rc"; tail -2 gpurun_out/bench_gloo2.log
