cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model bert --steps 10 --warmup 3 --eager-compare 0 --recall 0 > gpurun_out/bb.log 2>&1; rc=$?; tail -1 gpurun_out/bb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model bert --batch 256 --steps 5 --warmup 2 --eager-compare 0 --recall 0 > gpurun_out/bb256.log 2>&1; rc=$?; tail -1 gpurun_out/bb256.log
