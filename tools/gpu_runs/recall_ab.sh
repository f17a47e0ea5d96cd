# Recall@10 quality guard with and without the query side stream (training nondeterminism
# vs a cross-stream race): two runs each.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for qs in 1 0; do
    PAGEVEC_QUERY_STREAM=$qs timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -s --timeout 150 --timeout-method thread -k "recall_quality" > gpurun_out/rq_$qs_$r.log 2>&1
    echo "qs=$qs run=$r rc=$? $(grep -o 'recall@10 after 1000 steps: [0-9.]*' gpurun_out/rq_$qs_$r.log)"
  done
done
