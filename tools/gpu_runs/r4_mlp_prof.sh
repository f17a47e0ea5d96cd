cd $GRAFT_REPO_ROOT
M=${M:-mlp}
mkdir -p gpurun_out/r4_$M
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4_$M/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model $M --steps 20 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r4_$M/prof.log 2>&1
echo "prof rc=$?"
