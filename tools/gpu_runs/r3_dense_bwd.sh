# Round 3: dense backward GEMMs, library vs in-tree kernels (tools/dense_bwd_micro.py)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbwd
timeout -k 10 300 python3 tools/dense_bwd_micro.py > gpurun_out/dbwd/micro.log 2>&1
rc=$?; cat gpurun_out/dbwd/micro.log; exit $rc
