# Column-sum kernel + fused bag bias/activation: GPU tests, MLP A/B vs the previous commit's
# numbers (printed), BERT and chunked benches.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "colsum or embedding_bag or mlp or direct or hipgraph or linear or qkv or big_model or fp8" > gpurun_out/colsum_tests.log 2>&1
rc=$?; tail -3 gpurun_out/colsum_tests.log; [ $rc -eq 0 ] || exit $rc
for m in mlp chunked bert; do
  S=30; [ $m = bert ] && S=10
  timeout -k 10 200 python bench.py --model $m --steps $S --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0 > gpurun_out/cs_$m.log 2>&1 || exit 1
  echo "$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/cs_$m.log)"
done
