cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_flags
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag EARLY_SORT_SKIP --preset longpage_cdssm > gpurun_out/r4_flags/ess_ch.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/ess_ch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag EARLY_SORT_SKIP > gpurun_out/r4_flags/ess_head.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/ess_head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag EARLY_SORT_SKIP --preset reference_char --set dtype=bf16 --set vocab_hash_size=100 --set batch_size=1024 --set loss_mode=explicit > gpurun_out/r4_flags/ess_char.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/ess_char.log; exit $rc
