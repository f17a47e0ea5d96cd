# which part of the row-sparse CDSSM arm makes two EAGER runs diverge
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_sparse
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 240 python tools/sparse_graph_diag.py --runs e,e,e "$@" > $O/$tag.log 2>&1 || exit $?; echo "== $tag"; grep "config\|run [12]" $O/$tag.log; }
run sparse_lazy
run dense_lazy --set sparse_embedding_grad=false
run dense_nolazy --set sparse_embedding_grad=false --set lazy_embedding_adam=false
run sparse_lazy_noqstream --set query_stream=false
PAGEVEC_FORCE_DIST=0 run sparse_lazy_noexchange
PAGEVEC_STEP_PRIORITY=0 run sparse_lazy_noprio
