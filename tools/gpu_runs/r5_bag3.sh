# bag_gemm.hip: numerics, micro, kernel stats of the micro (per-kernel times of the list builder)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_bag3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bag_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_bag3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r5_bag3/pytest.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/r5_bag3/pytest.log; exit $rc; }
timeout -k 10 200 python tools/bag_gemm_micro.py > gpurun_out/r5_bag3/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; tail -1 gpurun_out/r5_bag3/micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_bag3/prof -- python3 tools/bag_gemm_micro.py > gpurun_out/r5_bag3/prof.log 2>&1
echo "prof rc=$?"
