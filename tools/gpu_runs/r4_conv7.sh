# Round 4: conv forward v7 (role-split: 8 MFMA waves + 4 loader waves) vs v4 -- bit identity + timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_conv7
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "role_split or conv_pool_fwd_bwd" > gpurun_out/r4_conv7/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r4_conv7/tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/conv_micro.py --variants 4096,16453,24645,24644,24641,24709,25669 --rounds 5 > gpurun_out/r4_conv7/conv_micro.log 2>&1
rc=$?; grep '^{' gpurun_out/r4_conv7/conv_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r4_conv7/bench_v4.log 2>&1
rc=$?; echo "bench v4 rc=$rc $(tail -1 gpurun_out/r4_conv7/bench_v4.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
PAGEVEC_CONV_DBG=24645 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r4_conv7/bench_v7.log 2>&1
rc=$?; echo "bench v7 rc=$rc $(tail -1 gpurun_out/r4_conv7/bench_v7.log | cut -c1-200)"; exit $rc
