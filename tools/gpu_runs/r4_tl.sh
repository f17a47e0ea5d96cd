# Round 4: kernel trace of the headline step -> one-step timeline + stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_tl
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_tl/prof -o cdssm -- python3 bench.py --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r4_tl/prof.log 2>&1
rc=$?; echo "prof rc=$rc $(grep '^{' gpurun_out/r4_tl/prof.log | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
python3 tools/timeline.py gpurun_out/r4_tl/prof/cdssm_kernel_trace.csv > gpurun_out/r4_tl/timeline.txt
python3 tools/prof_summary.py gpurun_out/r4_tl/prof/cdssm_kernel_stats.csv --steps 23 --top 30 --title "cdssm kernel stats (round 4, early sort)" > gpurun_out/r4_tl/cdssm_stats.md
cat gpurun_out/r4_tl/timeline.txt
for i in 1 2; do
timeout -k 10 300 python -u bench.py --quality-steps 0 --recall 0 --eager-compare 0 --steps 30 > gpurun_out/r4_tl/bench_$i.log 2>&1
rc=$?; echo "bench rc=$rc $(grep '^{' gpurun_out/r4_tl/bench_$i.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
done
