cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/ib_micro.py > gpurun_out/ib_micro.log 2>&1; rc=$?; cat gpurun_out/ib_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --eager-compare 0 > gpurun_out/b.log 2>&1; rc=$?; tail -1 gpurun_out/b.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ibprof3 -o ib -- python3 $GRAFT_REPO_ROOT/tools/ib_micro.py --M 16384,131072 --iters 5 > /dev/null 2>&1; echo prof rc=$?
