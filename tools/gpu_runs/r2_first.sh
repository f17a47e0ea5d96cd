# Round 2, first GPU pass: GPU tests, headline bench, then the hipGraph fault probe (last:
# it may fault, and nothing runs on the GPU after it).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -3
[ $rc -eq 0 ] || exit $rc
# probe: graph replays WITHOUT the per-replay fence, fresh batches each step, eval (eager
# encode) at step 100 -- the round-1 fault appeared after ~97 replays
timeout -k 10 240 python -u tools/quality_run.py --graph 1 --graph-fence 0 --batch 512 --steps 130 --eval-every 100 \
   --no-initial-eval --print-each > gpurun_out/graph_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids gpurun_out/graph_probe.log | tail -12
exit $rc
