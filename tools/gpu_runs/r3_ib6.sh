# Round 3: 4-wave workgroups (version 6) vs 8-wave (5): tests + ib_micro + kernel trace at the W = 8 shape
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ib6
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "inbatch_loss_split" > gpurun_out/ib6/tests.log 2>&1
rc=$?; tail -3 gpurun_out/ib6/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ib_micro.py --M 16384,131072 --iters 10 --ib 5,6,3,5,6 > gpurun_out/ib6/time.log 2>&1
rc=$?; cat gpurun_out/ib6/time.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ib6/kt -o kt -- python3 tools/ib_micro.py --M 131072 --iters 3 --ib 5,6 > gpurun_out/ib6/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; exit $rc
