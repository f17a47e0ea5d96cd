# Round 3: multi-rank GPU tests (query side stream under DDP, wide-vector cross-GPU loss)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_distributed_gpu.py > gpurun_out/dist/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error" gpurun_out/dist/tests.log | cut -c1-160; tail -3 gpurun_out/dist/tests.log; exit $rc
