# Round 3: ib5 at DP = 128 (MLP towers): tests + ib_micro at the W = 8 shape
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ib128
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "inbatch_loss_split" > gpurun_out/ib128/tests.log 2>&1
rc=$?; tail -3 gpurun_out/ib128/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ib_micro.py --D 128 --M 16384,131072 --iters 10 --ib 5,3,2,5,3 > gpurun_out/ib128/time.log 2>&1
rc=$?; cat gpurun_out/ib128/time.log; exit $rc
