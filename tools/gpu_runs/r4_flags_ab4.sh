cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_flags
timeout -k 10 200 python -u tools/step_flag_ab.py --setter pv_conv_set_dbg --vals 0,17541 > gpurun_out/r4_flags/pf2.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/pf2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/step_flag_ab.py --setter pv_conv_set_dbg --vals 0,17605 > gpurun_out/r4_flags/pf3.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/pf3.log; exit $rc
