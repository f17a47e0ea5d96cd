cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_flags
for F in EARLY_SORT DW_SIDE_STREAM SIDE_PER_STREAM BIAS_SINK; do
timeout -k 10 200 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag $F > gpurun_out/r4_flags/$F.log 2>&1
rc=$?; grep "^{" gpurun_out/r4_flags/$F.log; [ $rc -eq 0 ] || exit $rc
done
