cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_ib
timeout -k 10 200 python -u tools/ib_micro.py --M 131072 > gpurun_out/r4_ib/micro.log 2>&1
rc=$?; grep "^ib" gpurun_out/r4_ib/micro.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4_ib/prof -o ib -- python3 $GRAFT_REPO_ROOT/tools/ib_micro.py --M 131072 --ib 3 --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/r4_ib/prof.log 2>&1
echo "prof rc=$?"
