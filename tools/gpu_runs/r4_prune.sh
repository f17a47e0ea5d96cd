# Round 4: after pruning reduce4/5/6 + the rocPRIM / counting sorts: the conv backward, sort
# and graph tests, the reduce7 key-width / occupancy micro, one headline bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_prune
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "dtable or radix_sort or word_vocab or emitted_keys or hipgraph or conv_pool_bwd or determin or inbatch or cross_gpu" > gpurun_out/r4_prune/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_prune/pytest.log)"; grep -E "FAILED|Error" gpurun_out/r4_prune/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/reduce_ab.py --rounds 5 > gpurun_out/r4_prune/reduce_ab.log 2>&1
rc=$?; echo "reduce_ab rc=$rc"; grep '^{' gpurun_out/r4_prune/reduce_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --quality-steps 0 --steps 30 > gpurun_out/r4_prune/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(grep '^{' gpurun_out/r4_prune/bench.log | cut -c1-260)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ib_micro.py --M 131072 > gpurun_out/r4_prune/ib_micro.log 2>&1
rc=$?; echo "ib_micro rc=$rc"; grep -v amdgpu.ids gpurun_out/r4_prune/ib_micro.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_prune/prof -o cdssm -- python3 bench.py --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r4_prune/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py gpurun_out/r4_prune/prof/cdssm_kernel_stats.csv --steps 23 --top 30 --title "cdssm kernel stats (round 4, after pruning)" > gpurun_out/r4_prune/cdssm_stats.md; exit $?
