# Conv forward chunk-size variants (tools/conv_variant_build.py): numerics + same-box timing.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/conv_R.log
for V in default 96 128 144 default; do
  if [ $V = default ]; then L=""; else L=$PWD/dnn_page_vectors_amd/lib/variants/libpagevec_hip_PV_CONV_R_$V.so; fi
  PAGEVEC_HIP_LIB=$L timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv_pool_fwd_bwd" > gpurun_out/pytest_R$V.log 2>&1
  rc=$?; echo "R=$V pytest rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/pytest_R$V.log; exit $rc; }
  echo "R=$V" >> gpurun_out/conv_R.log
  PAGEVEC_HIP_LIB=$L timeout -k 10 200 python tools/conv_micro.py --variants 0 --rounds 3 >> gpurun_out/conv_R.log 2>&1
  rc=$?; echo "R=$V micro rc=$rc $(tail -1 gpurun_out/conv_R.log)"; [ $rc -eq 0 ] || exit $rc
done
