# Round 3: conv bias gradient straight into the flat gradient vs autograd accumulation, same box, interleaved
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bab
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 1 0; do
    PAGEVEC_BIAS_SINK=$v timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/bab/$v.$r.log 2>&1
    rc=$?; echo "sink=$v $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bab/$v.$r.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
