cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "layernorm or bert or hipgraph or bias_grad or gelu" > gpurun_out/pytest_bert2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_bert2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model bert > gpurun_out/bench_bert.log 2>&1
rc=$?; echo "bert rc=$rc"; tail -1 gpurun_out/bench_bert.log
