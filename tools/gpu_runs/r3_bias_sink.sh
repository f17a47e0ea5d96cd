# Round 3: conv bias gradients written straight into the flat gradient (no cat backward / fill / adds):
# conv, determinism, DDP and training tests, then the headline bench twice
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bsink
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_kernels_gpu.py tests/test_distributed_gpu.py tests/test_determinism.py \
  -k "conv or cdssm or determin or ddp or grad or train or char or chunk" > gpurun_out/bsink/tests.log 2>&1
rc=$?; tail -3 gpurun_out/bsink/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/bsink/b$r.log 2>&1
  rc=$?; echo "bench $r: $(tail -1 gpurun_out/bsink/b$r.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
done
