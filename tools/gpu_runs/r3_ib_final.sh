# Round 3: loss-kernel generation 5 (default) validation: numerics tests (incl. the multi-rank
# cross-GPU loss on one GPU), ib_micro A/B, the headline bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ibf
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_distributed_gpu.py -k "inbatch or explicit or cross_gpu" > gpurun_out/ibf/tests.log 2>&1
rc=$?; tail -4 gpurun_out/ibf/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ib_micro.py --M 16384,131072 --iters 10 --ib 5,3,2,5,3 > gpurun_out/ibf/time.log 2>&1
rc=$?; cat gpurun_out/ibf/time.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/ibf/bench.log 2>&1
rc=$?; tail -2 gpurun_out/ibf/bench.log; exit $rc
