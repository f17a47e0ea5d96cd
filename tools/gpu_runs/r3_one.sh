# Round 3: cached backward seed (no ones fill per step): trainer / graph / training tests + headline bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/one
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_kernels_gpu.py tests/test_determinism.py tests/test_distributed_gpu.py \
  -k "train or graph or cdssm or determin or ddp or big_model or recall" > gpurun_out/one/tests.log 2>&1
rc=$?; tail -2 gpurun_out/one/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/one/bench.log 2>&1
rc=$?; echo "bench: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"recall_at_10": [0-9.]*' gpurun_out/one/bench.log | tr '\n' ' ')"; exit $rc
