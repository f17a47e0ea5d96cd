# Round 6: loss-glue batch statistics by a one-workgroup final kernel vs the last-workgroup
# ticket (agent-scope fences): tests, kernel stats, same-process A/B on the headline and MLP steps.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_glue3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "inbatch or cross or loss or sumsq or ib or adam" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cdssm -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof_cdssm.log 2>&1 || exit $?
f=$(find $O/prof_cdssm -name "*kernel_stats.csv" | head -1); t=$(find $O/prof_cdssm -name "*kernel_trace.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "cdssm step kernels (round 6, glue stats kernel)" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0" > $O/stats_cdssm.md && python tools/timeline.py $t > $O/timeline_cdssm.txt || exit 1
grep -E "ib_fin|ib_stats|sumsq|FillFun" $O/stats_cdssm.md | cut -c1-110
for preset in cdssm_ngram_bf16 mlp_xgpu; do
  timeout -k 10 300 python tools/step_flag_ab.py --setter pv_ib_fin_set_ticket --vals 0,1 --rounds 8 --preset $preset > $O/ab_ticket_$preset.json 2>$O/ab_ticket_$preset.err || exit $?
  cat $O/ab_ticket_$preset.json
done
