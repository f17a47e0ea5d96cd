cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_f32_prof
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4_f32_prof -o bwd -- python3 $GRAFT_REPO_ROOT/tools/f32_micro.py --bwd 1 --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/r4_f32_prof/bwd.log 2>&1
echo "prof rc=$?"
