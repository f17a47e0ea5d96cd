# Round 4: dropout keep-bit plane from the forward for the dW kernel (PAGEVEC_MASK_PLANE)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_mask
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "mask_plane or conv_pool or role_split or emitted_keys or dtable or determin" > gpurun_out/r4_mask/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_mask/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/reduce_ab.py --rounds 5 > gpurun_out/r4_mask/rab.log 2>&1
rc=$?; echo "reduce_ab rc=$rc $(grep '"dw"' gpurun_out/r4_mask/rab.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/conv_micro.py --variants 0 --rounds 3 > gpurun_out/r4_mask/conv.log 2>&1
rc=$?; echo "conv_micro rc=$rc $(grep fwd_ms gpurun_out/r4_mask/conv.log | tail -2)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for mp in 0 1; do
PAGEVEC_MASK_PLANE=$mp timeout -k 10 300 python -u bench.py --quality-steps 0 --recall 0 --eager-compare 0 --steps 40 > gpurun_out/r4_mask/b_${mp}_$i.log 2>&1
rc=$?; echo "bench mask_plane=$mp rc=$rc $(grep '^{' gpurun_out/r4_mask/b_${mp}_$i.log | cut -c100-175)"; [ $rc -eq 0 ] || exit $rc
done; done
