# reduce5 vs reduce7 (compile-time dropout mode + packed FMAs), kernel A/B then the headline step.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r7
export TMPDIR=/tmp
timeout -k 10 200 python tools/reduce_ab.py --rb "" > gpurun_out/r7/ab.log 2>&1
rc=$?; tail -3 gpurun_out/r7/ab.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 5 7; do
    PAGEVEC_REDUCE_V=$v timeout -k 10 300 python bench.py --recall 0 --eager-compare 0 --quality-steps 0 --steps 40 > gpurun_out/r7/b_${v}_$i.log 2>&1
    rc=$?; echo "reduce_v=$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r7/b_${v}_$i.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
