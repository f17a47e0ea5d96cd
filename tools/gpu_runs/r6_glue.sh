# Round 6: loss-glue fusion tests, the high-priority step stream A/B, a kernel timeline.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_glue
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "inbatch or loss or rccl or hipgraph" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.train.trainer --flag STEP_PRIORITY --rounds 8 > $O/prio_ab.log 2>&1 || exit $?
tail -1 $O/prio_ab.log
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.loss --flag FUSED_GLUE --rounds 8 > $O/glue_ab.log 2>&1 || exit $?
tail -1 $O/glue_ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof.log 2>&1 || exit $?
t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/timeline.py $t > $O/timeline.txt && tail -1 $O/prof.log | cut -c1-150 && tail -1 $O/timeline.txt
