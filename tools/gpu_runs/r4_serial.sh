# Round 4: kernel stats with every side stream off (serial kernels: per-kernel times without contention)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_serial
export TMPDIR=/tmp
export PAGEVEC_DW_STREAM=0 PAGEVEC_QUERY_STREAM=0 PAGEVEC_EARLY_SORT=0
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_serial/prof -o cdssm -- python3 bench.py --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r4_serial/prof.log 2>&1
rc=$?; echo "prof rc=$rc $(grep '^{' gpurun_out/r4_serial/prof.log | cut -c100-175)"; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py gpurun_out/r4_serial/prof/cdssm_kernel_stats.csv --steps 23 --top 30 --title "cdssm kernel stats, side streams off (serial)" > gpurun_out/r4_serial/cdssm_stats.md
python3 tools/timeline.py gpurun_out/r4_serial/prof/cdssm_kernel_trace.csv > gpurun_out/r4_serial/timeline.txt
head -16 gpurun_out/r4_serial/cdssm_stats.md
