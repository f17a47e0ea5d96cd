cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_flags
for F in EARLY_SORT SIDE_PER_STREAM DENSE_DX; do
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag $F --preset longpage_cdssm > gpurun_out/r4_flags/ch_$F.log 2>&1; rc=$?; grep "^{" gpurun_out/r4_flags/ch_$F.log; [ $rc -eq 0 ] || exit $rc
done
