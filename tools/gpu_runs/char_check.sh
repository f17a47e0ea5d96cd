# Char-level (reference default) conv numerics + bench, and the host featurizer benchmark.
#   gpurun -- 'bash tools/gpu_runs/char_check.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv_pool" > gpurun_out/pytest_char.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_char.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model cdssm_char > gpurun_out/bench_cdssm_char.log 2>&1
rc=$?; echo "cdssm_char rc=$rc"; tail -1 gpurun_out/bench_cdssm_char.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/featurize_bench.py --pages 4000 --threads 16 > gpurun_out/featurize_bench.log 2>&1
rc=$?; echo "featurize rc=$rc"; cat gpurun_out/featurize_bench.log
