# Round 6: same-process A/B of the high-priority step stream (trainer.STEP_PRIORITY), then a
# kernel timeline with it on.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_prio
mkdir -p $O
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.train.trainer --flag STEP_PRIORITY --rounds 8 > $O/ab.log 2>&1 || exit $?
tail -1 $O/ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof.log 2>&1 || exit $?
t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/timeline.py $t > $O/timeline.txt && grep -n "reduce7\|dw_kernel\|colsum\|step span" $O/timeline.txt
