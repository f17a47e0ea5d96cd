cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -k "hipgraph or adam" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for m in cdssm mlp chunked bert; do
timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --eager-compare 0 --recall 0 --graph 1 > gpurun_out/g_$m.log 2>&1; rc=$?; echo "$m graph rc=$rc"; tail -1 gpurun_out/g_$m.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --eager-compare 0 --recall 0 --graph 0 > gpurun_out/e_$m.log 2>&1; rc=$?; echo "$m eager rc=$rc"; tail -1 gpurun_out/e_$m.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
