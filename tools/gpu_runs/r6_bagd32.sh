# Round 6: bagd_mm_kernel with 32-deep K-steps and a 6-slot ring (5 steps in flight) vs 64-deep /
# 3 slots: numerics at both depths, the micro, and (with the winner) the MLP bench protocol.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_bagd32
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bag_gemm_gpu.py -x -v --timeout 100 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bag_gemm_micro.py > $O/micro.log 2>&1 || exit $?
tail -1 $O/micro.log
