# bag_gemm.hip: numerics tests, then the MLP / chunked benches and an MLP kernel profile.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_bag
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bag_gemm_gpu.py tests/test_kernels_gpu.py -k "bag or embedding or mlp or big_model or hipgraph_step" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_bag/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r5_bag/pytest.log)"; [ $rc -eq 0 ] || { tail -60 gpurun_out/r5_bag/pytest.log; exit $rc; }
for M in mlp chunked; do
  for A in hip lib; do
    PAGEVEC_BAG_GEMM=$A timeout -k 10 300 python bench.py --model $M --eager-compare 0 --quality-steps 0 --recall 0 > gpurun_out/r5_bag/bench_${M}_$A.log 2>&1
    rc=$?; echo "$M $A rc=$rc $(tail -1 gpurun_out/r5_bag/bench_${M}_$A.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_bag/prof_mlp -- python3 bench.py --model mlp --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r5_bag/prof_mlp.log 2>&1
echo "prof rc=$?"
timeout -k 10 180 ./tools/bin/mfma_micro > gpurun_out/r5_bag/mfma4.log 2>&1; echo "mfma rc=$?"; cat gpurun_out/r5_bag/mfma4.log
