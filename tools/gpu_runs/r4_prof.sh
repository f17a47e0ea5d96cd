# Round 4: kernel stats of the headline step (and optionally other models) with the current defaults
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_prof
export TMPDIR=/tmp
for M in ${MODELS:-cdssm}; do
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_prof/$M -o $M -- python3 bench.py --model $M --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r4_prof/$M.log 2>&1
rc=$?; echo "$M rc=$rc $(tail -1 gpurun_out/r4_prof/$M.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py gpurun_out/r4_prof/$M/${M}_kernel_stats.csv --steps 23 --top 30 --title "$M kernel stats (round 4)" > gpurun_out/r4_prof/${M}_stats.md
done
