# Round 3: counting sort + conv v5 (one wave per SIMD) A/B, then the bench with each sort
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "count_sort or radix_sort or conv_pool_fwd_bwd or hipgraph or big_model" > gpurun_out/r3b/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r3b/pytest.log)"; [ $rc -le 1 ] || exit $rc  # test failures: keep going
timeout -k 10 200 python tools/sort_micro.py --iters 30 --ipt 16 > gpurun_out/r3b/sort_micro.log 2>&1
rc=$?; echo "sort rc=$rc"; cat gpurun_out/r3b/sort_micro.log | grep '^{'; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_micro.py --variants 0,8192,8194,8195 --rounds 5 > gpurun_out/r3b/conv_micro.log 2>&1
rc=$?; echo "conv rc=$rc"; grep '^{' gpurun_out/r3b/conv_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --quality-steps 0 > gpurun_out/r3b/bench_csort.log 2>&1
rc=$?; echo "bench csort rc=$rc $(grep '^{' gpurun_out/r3b/bench_csort.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
PAGEVEC_SORT=rsort timeout -k 10 300 python bench.py --quality-steps 0 > gpurun_out/r3b/bench_rsort.log 2>&1
rc=$?; echo "bench rsort rc=$rc $(grep '^{' gpurun_out/r3b/bench_rsort.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3b/bench_csort2.log 2>&1
rc=$?; echo "bench csort2 rc=$rc $(grep '^{' gpurun_out/r3b/bench_csort2.log | cut -c1-300)"; exit $rc
