# Conv backward / forward timings + the conv numerics tests (after kernel changes).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv or hipgraph or cdssm or layernorm or debug" > gpurun_out/pytest_bwdab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_bwdab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bwd_micro.py --epw 512 --rounds 3 > gpurun_out/bwd_ab.log 2>&1 && timeout -k 10 200 python tools/conv_micro.py --variants 0 --rounds 3 >> gpurun_out/bwd_ab.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -E "emit|fwd_ms" gpurun_out/bwd_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --quality-steps 0 --eager-compare 0 > gpurun_out/bench_ab.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_ab.log | cut -c1-200
