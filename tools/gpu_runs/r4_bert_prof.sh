cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_bert
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4_bert/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model bert --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r4_bert/prof.log 2>&1
echo "prof rc=$?"
