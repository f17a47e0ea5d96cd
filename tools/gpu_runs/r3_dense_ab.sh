# Round 3: dense backward on the in-tree kernels: numerics + training tests, bench A/B vs the library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dab
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "linear_act or dense_backward or big_model or recall_quality or training_curve or mlp" > gpurun_out/dab/tests.log 2>&1
rc=$?; tail -4 gpurun_out/dab/tests.log; [ $rc -eq 0 ] || exit $rc
for m in mlp cdssm; do
  for v in hip lib hip; do
    PAGEVEC_DENSE_BWD=$v timeout -k 10 300 python3 bench.py --model $m --steps 30 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/dab/$m.$v.log 2>&1
    rc=$?; echo "$m $v: $(tail -1 gpurun_out/dab/$m.$v.log | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
  done
done
