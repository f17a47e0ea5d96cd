cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider -k "conv or train" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python tools/conv_micro.py --variants 0 --rounds 3 --bwd > gpurun_out/micro.log 2>&1; echo "micro rc=$?"; cat gpurun_out/micro.log | grep variant
grep bwd gpurun_out/micro.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench.log
