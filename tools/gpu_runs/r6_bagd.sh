# Round 6: dense-count in-tree bag GEMMs (bag_gemm.hip bagd_mm_kernel): numerics, the micro vs the
# library plan, and the MLP step A/B (lib vs dense) in one process.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_bagd
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bag_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bag_gemm_micro.py > $O/micro.log 2>&1 || exit $?
tail -1 $O/micro.log
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.embedding --flag BAG_GEMM --vals "'lib','dense'" --rounds 10 --preset mlp_xgpu > $O/ab_mlp.json 2>$O/ab_mlp.err || exit $?
cat $O/ab_mlp.json
