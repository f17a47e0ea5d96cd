# Kernel stats of one model's step (rocprofv3 kernel trace + stats only; no counters here).
# usage: r5_prof.sh <model> [extra bench args]
cd $GRAFT_REPO_ROOT
m=$1; shift
mkdir -p gpurun_out/r5_prof/$m
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5_prof/$m -o $m -- python3 $GRAFT_REPO_ROOT/bench.py --model $m --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 "$@" > $GRAFT_REPO_ROOT/gpurun_out/r5_prof/$m/bench.log 2>&1
rc=$?; echo "prof $m rc=$rc $(tail -1 $GRAFT_REPO_ROOT/gpurun_out/r5_prof/$m/bench.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r5_prof/$m -name "*kernel_stats.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "$m step kernels (round 5)" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --model $m --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 $*" > gpurun_out/r5_prof/${m}_kernel_stats_r5.md
echo "summary rc=$?"; head -12 gpurun_out/r5_prof/${m}_kernel_stats_r5.md
