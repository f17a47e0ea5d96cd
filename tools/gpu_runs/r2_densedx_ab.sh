# Query-tower table gradient: dense dX rows (default) vs the emit / sort / reduce7 path.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ddx
export TMPDIR=/tmp
for i in 1 2; do
  for v in 1 0; do
    PAGEVEC_DENSE_DX=$v timeout -k 10 300 python bench.py --recall 0 --eager-compare 0 --quality-steps 0 --steps 40 > gpurun_out/ddx/b_${v}_$i.log 2>&1
    rc=$?; echo "dense_dx=$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ddx/b_${v}_$i.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv_pool_fwd_bwd or dtable" > gpurun_out/ddx/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/ddx/pytest.log)"; exit $rc
