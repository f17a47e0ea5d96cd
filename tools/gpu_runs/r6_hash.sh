# Round 6: the full GPU suite on the new dropout group hash, then the headline bench (with its
# 1000-step quality phase) three times, then one kernel-stats profile.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_hash
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || exit $?
  tail -1 $O/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['recall_at_10'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "cdssm step kernels (round 6, new mask hash)" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0" > $O/stats.md && python tools/timeline.py $t > $O/timeline.txt && head -12 $O/stats.md && tail -1 $O/timeline.txt
