# Sparse embedding-bag backward (MLP query tower): GPU tests, then same-box A/B of
# PAGEVEC_BAG_SPARSE_BWD=0 (counts GEMM) vs default on the MLP bench, and an EPW sweep.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "embedding_bag or mlp or direct or hipgraph or radix or dense_dx or dtable or conv_pool" > gpurun_out/bag_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bag_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --model mlp --steps 30 --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0"
for r in 1 2; do
  timeout -k 10 200 env PAGEVEC_BAG_SPARSE_BWD=0 $B > gpurun_out/bag_a$r.log 2>&1 || exit 1
  timeout -k 10 200 $B > gpurun_out/bag_b$r.log 2>&1 || exit 1
  echo "A(counts) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bag_a$r.log)  B(sparse) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bag_b$r.log)"
done
for e in 32; do
  timeout -k 10 200 env PAGEVEC_BAG_EPW=$e $B > gpurun_out/bag_e$e.log 2>&1 || exit 1
  echo "EPW=$e $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bag_e$e.log)"
done
