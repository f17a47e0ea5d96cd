# Round 5 validation: (a) full GPU suite + smoke + the headline bench; (b) one bench line per
# other model.   usage: r5_final.sh a|b
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_final
export TMPDIR=/tmp
o=gpurun_out/r5_final
models="mlp chunked chunked_cdssm bert cdssm_char"
if [ "$1" = "a" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $o/pytest.log)"; grep -E "FAILED|Error" $o/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $o/smoke.log)"; [ $rc -eq 0 ] || exit $rc
models="cdssm"
fi
for M in $models; do
timeout -k 10 400 python -u bench.py --model $M > $o/bench_$M.log 2>&1
rc=$?; echo "bench $M rc=$rc $(grep '^{' $o/bench_$M.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], d.get("recall_at_10"))')"; [ $rc -eq 0 ] || exit $rc
done
