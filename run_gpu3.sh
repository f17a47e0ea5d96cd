cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1
echo "prof rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/prof2 -name "*.csv" | head
