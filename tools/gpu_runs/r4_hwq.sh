# Round 4: GPU_MAX_HW_QUEUES 8 vs the default 4 for the headline step (4 of our streams + RCCL's at W > 1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_hwq
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 300 python -u bench.py --quality-steps 0 --recall 0 --eager-compare 0 --steps 40 > gpurun_out/r4_hwq/b_4_$i.log 2>&1
rc=$?; echo "hwq=default rc=$rc $(grep '^{' gpurun_out/r4_hwq/b_4_$i.log | cut -c100-175)"; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u bench.py --quality-steps 0 --recall 0 --eager-compare 0 --steps 40 > gpurun_out/r4_hwq/b_8_$i.log 2>&1
rc=$?; echo "hwq=8 rc=$rc $(grep '^{' gpurun_out/r4_hwq/b_8_$i.log | cut -c100-175)"; [ $rc -eq 0 ] || exit $rc
done
