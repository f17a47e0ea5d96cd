# Same-box A/B of the headline: the round-5 tree (ab_r5/, built from 66ee3af) vs this tree,
# driver protocol without the quality phase, alternated 3x.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_vs_r5
mkdir -p $O
for i in 1 2 3; do
  (cd ab_r5 && PAGEVEC_NO_AUTOBUILD=1 timeout -k 10 300 python bench.py --recall 0 --quality-steps 0 --eager-compare 0 > $O/r5_$i.log 2>&1) || exit $?
  timeout -k 10 300 python bench.py --recall 0 --quality-steps 0 --eager-compare 0 > $O/r6_$i.log 2>&1 || exit $?
  echo "r5 $(tail -1 $O/r5_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")  r6 $(tail -1 $O/r6_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
