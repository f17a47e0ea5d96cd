# Round 6: the in-batch / cross-GPU loss at the headline (M 16384) and W = 8 (M 131072) shapes,
# fused finish kernels vs the round-5 glue launches, and a kernel-stats pass of the fused path.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_ibw8
mkdir -p $O
timeout -k 10 300 python tools/ib_micro.py --M 16384,131072 --ib 7 --glue 1,0 --iters 20 > $O/ib_micro.log 2>&1 || exit $?
grep "^ib" $O/ib_micro.log
#cd /tmp
#timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $GRAFT_REPO_ROOT/tools/ib_micro.py --M 131072 --ib 7 --glue 1 --iters 20 > $O/prof.log 2>&1 || exit $?
#f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
#cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 23 --title "in-batch loss at the W = 8 shape, fused glue (per fwd+bwd call)" --cmd "rocprofv3 --kernel-trace --stats -- python3 tools/ib_micro.py --M 131072 --ib 7 --glue 1 --iters 20" > $O/stats.md && head -16 $O/stats.md | cut -c1-150
for preset in cdssm_ngram_bf16 mlp_xgpu; do
  timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.loss --flag FUSED_GLUE --rounds 8 --preset $preset > $O/ab_glue_$preset.json 2>$O/ab_glue_$preset.err || exit $?
  cat $O/ab_glue_$preset.json
done
