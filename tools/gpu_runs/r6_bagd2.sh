# Round 6: dense-count in-tree bag GEMMs as the default: GPU tests of every bag / MLP / chunked /
# graph path, benches, the chunked fp8 A/B (its bf16 weight gradient), and the MLP kernel stats.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_bagd2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread -k "bag or mlp or chunk or graph or rccl or fp8 or embed" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for M in mlp chunked chunked_cdssm; do
timeout -k 10 300 python -u bench.py --model $M > $O/bench_$M.log 2>&1 || exit $?
grep '^{' $O/bench_$M.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], d["value"], d["ms_per_step"], d.get("recall_at_10"), d.get("graph_status"))'
done
timeout -k 10 300 python tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.embedding --flag BAG_GEMM --vals "'lib','auto'" --rounds 8 --preset mlp_xgpu > $O/ab_mlp_eager.json 2>$O/ab_mlp_eager.err || exit $?
cat $O/ab_mlp_eager.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o p -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof_mlp.log 2>&1 || exit $?
f=$(find $O/prof_mlp -name "*kernel_stats.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "mlp step kernels (round 6, in-tree dense-count bag GEMMs eager / library inside the graph)" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --model mlp --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0" > $O/stats_mlp.md && head -20 $O/stats_mlp.md | cut -c1-130
