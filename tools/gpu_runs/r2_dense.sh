# Round 2: dense-dX query backward: numerics vs the sort path, A/B timing, bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
   -k "dense_dx or conv_pool or cdssm_train or radix or unfenced" > gpurun_out/pytest_dense.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dense.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/qbwd_micro.py > gpurun_out/qbwd.log 2>&1
rc=$?; echo "qbwd rc=$rc"; grep -v amdgpu.ids gpurun_out/qbwd.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-400
exit $rc
