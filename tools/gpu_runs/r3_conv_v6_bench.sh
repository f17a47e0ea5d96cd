# Round 3: headline bench with the conv forward v4 (default) vs v6 (three waves per SIMD), same box, interleaved
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v6b
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 0 8236; do
    PAGEVEC_CONV_DBG=$v timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/v6b/$v.$r.log 2>&1
    rc=$?; echo "$v $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/v6b/$v.$r.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
