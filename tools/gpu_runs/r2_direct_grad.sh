# Direct flat-gradient writes (ops/grad_sink.py): GPU tests, then same-box A/B of
# PAGEVEC_DIRECT_GRAD=0 (autograd AccumulateGrad path) vs default, per model.
#   gpurun --timeout 900 -- 'bash tools/gpu_runs/r2_direct_grad.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "direct or train_step or qkv" \
  > gpurun_out/dg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dg_tests.log; [ $rc -eq 0 ] || exit $rc
for m in mlp cdssm bert; do
  S=30; [ $m = bert ] && S=10
  timeout -k 10 200 env PAGEVEC_DIRECT_GRAD=0 python bench.py --model $m --steps $S --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0 > gpurun_out/dg_a_$m.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --model $m --steps $S --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0 > gpurun_out/dg_b_$m.log 2>&1 || exit 1
  echo "$m A(off) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dg_a_$m.log)  B(on) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dg_b_$m.log)"
done
