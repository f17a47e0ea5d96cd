cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_flags
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag DW_SIDE_STREAM --preset longpage_cdssm > gpurun_out/r4_flags/dws_chunked.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/dws_chunked.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag DW_SIDE_STREAM --preset reference_char --set dtype=bf16 --set vocab_hash_size=100 --set batch_size=1024 --set loss_mode=explicit > gpurun_out/r4_flags/dws_char.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/dws_char.log; exit $rc
