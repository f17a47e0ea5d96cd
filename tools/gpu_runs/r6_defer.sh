# Round 6: the page tower's early table-gradient sort launched after the loss forward
# (PAGEVEC_DEFER_SORT): conv / graph / RCCL tests, same-process A/Bs, bench alternated.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_defer
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "conv or graph or rccl or determin or sparse or trainer" > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag DEFER_SORT --vals 0,2 --rounds 8 > $O/ab_02.json 2>$O/ab.err || exit $?
cat $O/ab_02.json
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag DEFER_SORT --vals 0,1 --rounds 8 --preset reference_char --set dtype=bf16 --set batch_size=1024 > $O/ab_char.json 2>>$O/ab.err || exit $?
cat $O/ab_char.json
for i in 1 2; do for v in 0 1; do
PAGEVEC_DEFER_SORT=$v timeout -k 10 300 python bench.py --recall 0 --quality-steps 0 --eager-compare 0 > $O/bench_${v}_$i.log 2>&1 || exit $?
echo "defer=$v $(tail -1 $O/bench_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
