# Round 6: re-measure the README's secondary numbers on the final tree — the deterministic
# headline step, page-vector extraction (encode) per model, and the serving top-k / engine.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_refresh
mkdir -p $O
timeout -k 10 300 python -u bench.py --deterministic 1 --recall 0 --quality-steps 0 --eager-compare 0 > $O/bench_det.log 2>&1 || exit $?
grep '^{' $O/bench_det.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("det", d["value"], d["ms_per_step"])'
for M in cdssm cdssm_char mlp bert; do
timeout -k 10 300 python -u tools/encode_bench.py --model $M > $O/encode_$M.log 2>&1 || exit $?
echo "encode $M $(tail -1 $O/encode_$M.log | cut -c1-200)"
done
timeout -k 10 300 python -u tools/serve_bench.py > $O/serve.log 2>&1 || exit $?
tail -3 $O/serve.log | cut -c1-300
