# Round 6 checkpoint: full GPU suite, smoke, the headline bench (driver protocol) x2
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || exit $?
  tail -1 $O/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['recall_at_10'], d['per_rank']['step_ms_rank_spread'], d['native_lib_stamp'])"
done
