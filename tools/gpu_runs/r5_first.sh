# Round 5 first look: MFMA shape micro, headline bench, one profiled step for the timeline.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_first
export TMPDIR=/tmp
timeout -k 10 120 ./tools/bin/mfma_micro > gpurun_out/r5_first/mfma.log 2>&1
rc=$?; echo "mfma rc=$rc"; cat gpurun_out/r5_first/mfma.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --eager-compare 0 > gpurun_out/r5_first/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(tail -1 gpurun_out/r5_first/bench.log | cut -c1-300)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5_first/prof -- python3 bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r5_first/prof.log 2>&1
echo "prof rc=$?"
