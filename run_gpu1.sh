cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python tools/conv_micro.py > gpurun_out/micro.log 2>&1
  echo "micro rc=$?"; cat gpurun_out/micro.log | tail -3
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
  rc=$?
  echo "bench rc=$rc"
  tail -3 gpurun_out/bench.log
fi
