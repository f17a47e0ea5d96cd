# Round 4: dW with the k = 3 pieces of 4 samples packed into 3 instructions (PAGEVEC_DW_PACK)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_dwpack
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv_pool or conv_backward or dw or determin or training_curve" > gpurun_out/r4_dwpack/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_dwpack/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for pk in 0 1; do
PAGEVEC_DW_PACK=$pk timeout -k 10 200 python -u tools/reduce_ab.py --rounds 5 > gpurun_out/r4_dwpack/rab_$pk.log 2>&1
rc=$?; echo "reduce_ab pack=$pk rc=$rc $(grep '"dw"' gpurun_out/r4_dwpack/rab_$pk.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do for pk in 0 1; do
PAGEVEC_DW_PACK=$pk timeout -k 10 300 python -u bench.py --quality-steps 0 --recall 0 --eager-compare 0 --steps 40 > gpurun_out/r4_dwpack/b_${pk}_$i.log 2>&1
rc=$?; echo "bench pack=$pk rc=$rc $(grep '^{' gpurun_out/r4_dwpack/b_${pk}_$i.log | cut -c100-175)"; [ $rc -eq 0 ] || exit $rc
done; done
