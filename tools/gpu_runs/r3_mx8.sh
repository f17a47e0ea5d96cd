# Round 3: MX fp8 GEMM numerics + micro-benchmark
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3mx
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -s -k "mx8 or counts8 or fp8_bag or mx_fp8" > gpurun_out/r3mx/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3mx/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mx8_micro.py > gpurun_out/r3mx/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/r3mx/micro.log | grep "{"; exit $rc
