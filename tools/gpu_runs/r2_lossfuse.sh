# Fused loss mean / accuracy / backward prologue: GPU tests, 2-rank gloo tests, rehearsal, benches.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_distributed_gpu.py \
  -k "loss or train_step or hipgraph or direct or ddp or cross_gpu" -m gpu > gpurun_out/lf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lf_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_runs/dist_rehearsal.sh || exit 1
for m in mlp cdssm; do
  timeout -k 10 200 python bench.py --model $m --steps 30 --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0 > gpurun_out/lf_$m.log 2>&1 || exit 1
  echo "$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lf_$m.log)"
done
