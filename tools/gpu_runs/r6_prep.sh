# Round 6: full GPU suite on the current tree (capture streams default on, sparse overflow flag,
# step priority, one-launch tower prep), smoke, then the one-launch tower prep A/B (same process,
# interleaved) and a kernel-trace timeline of the headline step.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_prep
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag PREP_MULTI --rounds 10 > $O/ab_cdssm.json 2>$O/ab_cdssm.err || exit $?
cat $O/ab_cdssm.json
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.conv_pool --flag PREP_MULTI --rounds 10 --preset longpage_cdssm > $O/ab_chunked.json 2>$O/ab_chunked.err || exit $?
cat $O/ab_chunked.json
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['recall_at_10'], d['native_lib_stamp'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "cdssm step kernels (round 6, one-launch tower prep)" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0" > $O/stats.md && python tools/timeline.py $t > $O/timeline.txt && tail -8 $O/timeline.txt
