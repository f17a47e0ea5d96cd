cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_flags
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag DENSE_DX > gpurun_out/r4_flags/densedx.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/densedx.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.grad_sink --flag ENABLED > gpurun_out/r4_flags/gradsink.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/gradsink.log; exit $rc
