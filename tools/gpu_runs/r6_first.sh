# Round 6 first box: baseline step, and the dropout-off step (upper bound of what a cheaper
# mask hash can save in the conv forward staging, dW and the dTable reduce).
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_first
mkdir -p $O
B="--steps 20 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0"
timeout -k 10 300 python bench.py $B > $O/bench_base.log 2>&1 || exit $?
tail -1 $O/bench_base.log | cut -c1-160
timeout -k 10 300 python bench.py $B --set 'dropout_prob=[0.0,0.5]' > $O/bench_nodrop.log 2>&1 || exit $?
tail -1 $O/bench_nodrop.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp
for arm in base nodrop; do
  extra=""; [ $arm = nodrop ] && extra="--set dropout_prob=[0.0,0.5]"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$arm -o $arm -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 $extra > $O/prof_$arm.log 2>&1 || exit $?
  f=$(find $O/prof_$arm -name "*kernel_stats.csv" | head -1)
  t=$(find $O/prof_$arm -name "*kernel_trace.csv" | head -1)
  (cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "cdssm $arm" --cmd "bench $arm" > $O/stats_$arm.md && python tools/timeline.py $t > $O/timeline_$arm.txt) || exit $?
  head -14 $O/stats_$arm.md
done
