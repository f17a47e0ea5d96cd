cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider -k "conv or train" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit 1
for d in 0 2 4 7; do
  PAGEVEC_CONV_DBG=$d timeout -k 10 120 python tools/conv_micro.py --iters 10 > gpurun_out/abl_$d.log 2>&1 || exit 1
  echo "dbg=$d $(tail -1 gpurun_out/abl_$d.log)"
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench.log
