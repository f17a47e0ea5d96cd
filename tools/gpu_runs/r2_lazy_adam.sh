# Lazy embedding-row Adam: GPU tests + micro benchmark (7.5M x 100 word table, 1% rows touched).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "adam or hipgraph" > gpurun_out/lazy_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lazy_tests.log; [ $rc -eq 0 ] || exit $rc
{ timeout -k 10 120 python tools/adam_micro.py --lazy-rows 7500000 --lazy-cols 100 --touched 0.01 && timeout -k 10 120 python tools/adam_micro.py --n 1024 --lazy-rows 1000000 --lazy-cols 300 --touched 0.05; } > gpurun_out/lazy_micro.log 2>&1
rc=$?; cat gpurun_out/lazy_micro.log | tail -2; exit $rc
