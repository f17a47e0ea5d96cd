# ADVICE r5 follow-up: first-run effect in the lazy-Adam arms (a throwaway trainer first), the
# RCCL test configuration eager vs graph over all 22 steps; then the conv forward micro with the
# round-5 vs round-6 dropout group hash (same process per library, alternated).
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_sparse2
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 240 python tools/sparse_graph_diag.py "$@" > $O/$tag.log 2>&1 || exit $?; echo "== $tag"; grep "run [1-3]" $O/$tag.log; }
run dense_lazy_burn --runs e,e,e --burn 1 --set sparse_embedding_grad=false
PAGEVEC_FORCE_DIST=0 run sparse_lazy_noexch_burn --runs e,e,e --burn 1
run sparse_lazy_eg --runs e,g,e,g
LEG=$GRAFT_REPO_ROOT/dnn_page_vectors_amd/lib/variants/libpagevec_hip_PV_DROP_HASH_LEGACY_1.so
for i in 1 2; do
  timeout -k 10 200 python tools/conv_micro.py --variants 0 --rounds 3 > $O/conv_new_$i.log 2>&1 || exit $?
  PAGEVEC_HIP_LIB=$LEG timeout -k 10 200 python tools/conv_micro.py --variants 0 --rounds 3 > $O/conv_legacy_$i.log 2>&1 || exit $?
  echo "new $(grep fwd_ms_median $O/conv_new_$i.log)"; echo "legacy $(grep fwd_ms_median $O/conv_legacy_$i.log)"
done
