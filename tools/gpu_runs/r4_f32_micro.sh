cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_f32_pmc
timeout -k 10 200 python -u -m pytest tests/test_conv_f32_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_f32_pmc/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_f32_pmc/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/f32_micro.py > gpurun_out/r4_f32_pmc/micro.log 2>&1
rc=$?; grep '^{' gpurun_out/r4_f32_pmc/micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/f32_micro.py --bwd 1 --iters 5 > gpurun_out/r4_f32_pmc/micro_bwd.log 2>&1
rc=$?; grep '^{' gpurun_out/r4_f32_pmc/micro_bwd.log; exit $rc
