# Round 4 validation: full GPU suite + smoke, then one bench line per model and kernel stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_final
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_final/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_final/pytest.log)"; grep -E "FAILED|Error" gpurun_out/r4_final/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_final/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/r4_final/smoke.log)"; [ $rc -eq 0 ] || exit $rc
for M in cdssm mlp chunked chunked_cdssm bert cdssm_char; do
timeout -k 10 400 python -u bench.py --model $M > gpurun_out/r4_final/bench_$M.log 2>&1
rc=$?; echo "bench $M rc=$rc $(grep '^{' gpurun_out/r4_final/bench_$M.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], d.get("recall_at_10"))')"; [ $rc -eq 0 ] || exit $rc
done
