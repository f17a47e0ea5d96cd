# Round 3: wide-vector (D = 768) in-batch loss tiled over page-column blocks: tests + BERT bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wide
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_distributed_gpu.py \
  -k "wide_rows or big_model or bert or inbatch" > gpurun_out/wide/tests.log 2>&1
rc=$?; tail -4 gpurun_out/wide/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --model bert --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/wide/bert.log 2>&1
rc=$?; echo "bert: $(tail -1 gpurun_out/wide/bert.log | cut -c1-200)"; exit $rc
