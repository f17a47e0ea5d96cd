# Kernel trace of the eager CDSSM step: GPU idle (host launch latency) per step.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gaps
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps/cdssm -- python3 bench.py --steps 8 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/gaps/cdssm.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/gaps/cdssm -name '*kernel_trace.csv' | head -1)
python3 tools/trace_gaps.py "$f" --top 10 > gpurun_out/gaps/cdssm_gaps.txt 2>&1; echo "gaps rc=$?"
tail -30 gpurun_out/gaps/cdssm_gaps.txt
