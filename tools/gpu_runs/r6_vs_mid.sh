# Same-box A/B of the headline: the mid-round-6 validation tree (ab_mid/, built from 3813d9e) vs this tree,
# driver protocol without the quality phase, alternated 3x.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_vs_mid
mkdir -p $O
for i in 1 2 3; do
  (cd ab_mid && PAGEVEC_NO_AUTOBUILD=1 timeout -k 10 300 python bench.py --recall 0 --quality-steps 0 --eager-compare 0 > $O/mid_$i.log 2>&1) || exit $?
  timeout -k 10 300 python bench.py --recall 0 --quality-steps 0 --eager-compare 0 > $O/head_$i.log 2>&1 || exit $?
  echo "mid $(tail -1 $O/mid_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")  head $(tail -1 $O/head_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
