# Round 3: bucketed table-gradient chain (one radix pass + reduce8 LDS accumulation) vs
# emit -> 2-pass sort -> reduce7: numerics tests, same-process chain A/B, headline bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r8
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "reduce8 or conv_pool_fwd_bwd or dtable_reduce" > gpurun_out/r8/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r8/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/table_chain_ab.py --rounds 5 > gpurun_out/r8/chain.log 2>&1
rc=$?; cat gpurun_out/r8/chain.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/table_chain_ab.py --N 4096 --L 45 --seg 4096,16384 --rounds 5 > gpurun_out/r8/chain_q.log 2>&1
rc=$?; cat gpurun_out/r8/chain_q.log; exit $rc
