# Round 2: conv forward A/B (same process): production v2 (0) vs v3 (512: compile-time
# dropout mode, 3 wave bodies) — bit-exactness check + timing; numerics test on v3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VARS=${VARS:-0,512}
timeout -k 10 300 python -u tools/conv_micro.py --variants $VARS --rounds 5 > gpurun_out/conv_ab.log 2>&1
rc=$?; echo "conv_micro rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_ab.log | tail -8
[ $rc -eq 0 ] || exit $rc
PAGEVEC_CONV_DBG=${TESTVAR:-512} timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
   -k "conv_pool" > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log
exit $rc
