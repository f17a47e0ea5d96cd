# Round 6: bench.py with and without the high-priority step stream, alternated on one box.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_prio2
mkdir -p $O
for i in 1 2 3; do
  for v in 0 1; do
    PAGEVEC_STEP_PRIORITY=$v timeout -k 10 300 python bench.py --recall 0 --quality-steps 0 --eager-compare 0 > $O/b_${v}_$i.log 2>&1 || exit $?
    echo "prio $v run $i $(tail -1 $O/b_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['per_rank']['step_ms_median_per_rank'])")"
  done
done
