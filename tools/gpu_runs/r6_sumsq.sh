# Round 6: the fill-free, deterministic gradient sum of squares (pv_sumsq_ticket): tests, then
# same-process interleaved A/B on the headline, MLP and chunked CDSSM eager steps.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_sumsq
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sumsq or adam or trainer or hipgraph or determin or sparse" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for preset in cdssm_ngram_bf16 mlp_xgpu longpage_cdssm; do
  timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.optim --flag SUMSQ_TICKET --rounds 10 --preset $preset > $O/ab_$preset.json 2>$O/ab_$preset.err || exit $?
  cat $O/ab_$preset.json
done
