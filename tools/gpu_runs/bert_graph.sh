# BERT hipGraph replay check + the BERT / chunked benches (the last bench_all run faulted in BERT).
#   gpurun --timeout 900 -- 'bash tools/gpu_runs/bert_graph.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "hipgraph or big_model or topk" > gpurun_out/pytest_graph.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_graph.log
[ $rc -eq 0 ] || exit $rc
for M in bert chunked; do
  timeout -k 10 300 python -u bench.py --model $M > gpurun_out/bench_$M.log 2>&1
  rc=$?; echo "$M rc=$rc"; tail -1 gpurun_out/bench_$M.log
  [ $rc -eq 0 ] || exit $rc
done
