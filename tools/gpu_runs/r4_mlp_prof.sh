cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_mlp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4_mlp/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 20 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r4_mlp/prof.log 2>&1
echo "prof rc=$?"
