# Round 6: the MLP headline protocol (graph-captured step) with the library vs the in-tree
# dense-count bag GEMMs, alternated 3x on one box.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_bagd3
mkdir -p $O
for i in 1 2 3; do
for arm in lib dense; do
PAGEVEC_BAG_GEMM=$arm timeout -k 10 300 python -u bench.py --model mlp --quality-steps 0 --recall 0 > $O/mlp_${arm}_$i.log 2>&1 || exit $?
echo "$arm $i $(grep '^{' $O/mlp_${arm}_$i.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("graph_status"))')"
done
done
