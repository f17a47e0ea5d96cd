# Round 3: side-stream dW enqueue point (before the table chain / after the sort / after the reduce), headline A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dwat
export TMPDIR=/tmp
for r in 1 2; do
  for v in first sort reduce; do
    PAGEVEC_DW_AT=$v timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/dwat/$v.$r.log 2>&1
    rc=$?; echo "$v $r: $(tail -1 gpurun_out/dwat/$v.$r.log | cut -c1-140)"; [ $rc -eq 0 ] || exit $rc
  done
done
