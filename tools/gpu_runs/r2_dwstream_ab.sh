# Headline step with the page dW kernel on a side stream (beside emit/sort/reduce) vs inline.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dws
export TMPDIR=/tmp
for i in 1 2; do
  for v in 0 1; do
    PAGEVEC_DW_STREAM=$v timeout -k 10 300 python bench.py --recall 0 --eager-compare 0 --quality-steps 0 --steps 40 > gpurun_out/dws/b_${v}_$i.log 2>&1
    rc=$?; echo "dw_stream=$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dws/b_${v}_$i.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
