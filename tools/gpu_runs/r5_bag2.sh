# bag_gemm.hip iteration: numerics, micro (in-tree vs library), MLP bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_bag2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bag_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_bag2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r5_bag2/pytest.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/r5_bag2/pytest.log; exit $rc; }
timeout -k 10 200 python tools/bag_gemm_micro.py > gpurun_out/r5_bag2/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; tail -2 gpurun_out/r5_bag2/micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bag_gemm_micro.py --L 512 > gpurun_out/r5_bag2/micro512.log 2>&1
rc=$?; echo "micro512 rc=$rc"; tail -1 gpurun_out/r5_bag2/micro512.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model mlp --eager-compare 0 --quality-steps 0 --recall 0 > gpurun_out/r5_bag2/bench_mlp.log 2>&1
rc=$?; echo "mlp rc=$rc $(tail -1 gpurun_out/r5_bag2/bench_mlp.log | cut -c1-200)"
