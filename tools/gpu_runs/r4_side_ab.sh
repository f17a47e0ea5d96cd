# Round 4: per-tower side streams vs one shared side stream (dW + early sort), interleaved
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_side
export TMPDIR=/tmp
for i in 1 2 3; do
for ps in 0 1; do
PAGEVEC_SIDE_PER_STREAM=$ps timeout -k 10 300 python -u bench.py --quality-steps 0 --recall 0 --eager-compare 0 --steps 40 > gpurun_out/r4_side/b_${ps}_$i.log 2>&1
rc=$?; echo "per_stream=$ps rc=$rc $(grep '^{' gpurun_out/r4_side/b_${ps}_$i.log | cut -c100-175)"; [ $rc -eq 0 ] || exit $rc
done; done
