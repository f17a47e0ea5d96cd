# Round 2: in-tree radix sort — numerics, A/B timing vs rocPRIM, bench, then the unfenced
# hipGraph probe that faulted with rocPRIM (last: nothing runs on the GPU after it).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
   -k "radix_sort or conv_pool or cdssm or hipgraph or dtable" > gpurun_out/pytest_sort.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_sort.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/sort_micro.py > gpurun_out/sort_micro.log 2>&1
rc=$?; echo "sort_micro rc=$rc"; grep -v amdgpu.ids gpurun_out/sort_micro.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/quality_run.py --graph 1 --graph-fence 0 --batch 512 --steps 300 --eval-every 100 \
   --no-initial-eval > gpurun_out/graph_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids gpurun_out/graph_probe.log | tail -6
exit $rc
