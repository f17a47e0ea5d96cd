# Round 6: loss-glue split sums with eight loads in flight, sumsq up to 2048 workgroups: loss /
# sumsq tests, then per-kernel stats of the headline and MLP steps.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_glue2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "inbatch or cross or loss or sumsq or ib" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for m in cdssm mlp; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o p -- python3 $GRAFT_REPO_ROOT/bench.py --model $m --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof_$m.log 2>&1 || exit $?
  f=$(find $O/prof_$m -name "*kernel_stats.csv" | head -1)
  (cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "$m step kernels (round 6, batched split sums)" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --model $m --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0" > $O/stats_$m.md) || exit 1
  grep -E "ib_fin|sumsq|split_reduce" $O/stats_$m.md | cut -c1-120
done
