cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/conv_micro.py --variants 0,36,128 --rounds 3 --bwd > gpurun_out/micro.log 2>&1; rc=$?; cat gpurun_out/micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --eager-compare 0 > gpurun_out/b.log 2>&1; rc=$?; tail -1 gpurun_out/b.log
