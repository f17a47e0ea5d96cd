# Round 6: conv GPU tests on the LDS-staged dW kernel, the headline step, then the dropout
# hash quality A/B (tools/gpu_runs/r6_hashq.sh).
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_dw
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "conv or dropout or cdssm or hipgraph or rccl" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --recall 0 --quality-steps 0 --eager-compare 0 > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "cdssm step kernels (round 6, LDS-staged dW)" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0" > $O/stats.md && python tools/timeline.py $t > $O/timeline.txt && head -12 $O/stats.md | tail -5 && tail -1 $O/timeline.txt || exit 1
bash tools/gpu_runs/r6_hashq.sh
