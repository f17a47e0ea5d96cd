# Round 6: kernel stats + timeline of the reference-default config (char CDSSM, L 5000, B 1024, bf16).
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_char_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --model cdssm_char --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "cdssm_char step kernels (round 6)" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --model cdssm_char --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0" > $O/stats.md && python tools/timeline.py $t > $O/timeline.txt && head -22 $O/stats.md | cut -c1-140 && tail -1 $O/timeline.txt
