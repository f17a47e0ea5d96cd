cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_flags
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag REDUCE_EPW --vals 512,256 > gpurun_out/r4_flags/epw256.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/epw256.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag REDUCE_EPW --vals 512,1024 > gpurun_out/r4_flags/epw1024.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/epw1024.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/step_flag_ab.py --setter pv_conv_r7_set_occ --vals 8,1 > gpurun_out/r4_flags/occ.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/occ.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/step_flag_ab.py --setter pv_rsort_set_ipt --vals 0,32 > gpurun_out/r4_flags/ipt32.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/ipt32.log; exit $rc
