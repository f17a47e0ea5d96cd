# Optimizer kernels: numerics + the configs where Adam / sumsq matter (mlp, chunked).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "adam or sumsq or hipgraph" > gpurun_out/pytest_optim.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_optim.log
[ $rc -eq 0 ] || exit $rc
for M in mlp chunked; do
  timeout -k 10 300 python -u bench.py --model $M --quality-steps 0 --recall 0 > gpurun_out/bench_$M.log 2>&1
  rc=$?; echo "$M rc=$rc $(tail -1 gpurun_out/bench_$M.log | cut -c1-200)"
  [ $rc -eq 0 ] || exit $rc
done
