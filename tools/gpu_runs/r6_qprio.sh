# Round 6: the query-tower stream at high priority (its forward sits between the page conv and
# the loss, beside the page tower's early sort): same-process A/B on the headline, then bench x2
# each way alternated.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_qprio
mkdir -p $O
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.models.base --flag QUERY_HIGH_PRIORITY --rounds 10 > $O/ab.json 2>$O/ab.err || exit $?
cat $O/ab.json
for i in 1 2; do for v in 0 1; do
PAGEVEC_QUERY_PRIORITY=$v timeout -k 10 300 python bench.py --recall 0 --quality-steps 0 --eager-compare 0 > $O/bench_${v}_$i.log 2>&1 || exit $?
echo "qprio=$v $(tail -1 $O/bench_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
