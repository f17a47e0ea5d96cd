# Round 6 validation: (a) full GPU suite + smoke + the headline bench x2 + the multi-rank
# rehearsal over gloo; (b) one bench line per other model (+ the reference-precision config).
#   usage: r6_final.sh a|b
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6_final
export TMPDIR=/tmp
o=gpurun_out/r6_final
bl() { grep '^{' $1 | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], d.get("recall_at_10"), d.get("graph_status"))'; }
if [ "$1" = "a" ]; then
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $o/pytest.log)"; grep -E "FAILED|Error" $o/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $o/smoke.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 400 python -u bench.py > $o/bench_cdssm_$i.log 2>&1
rc=$?; echo "bench cdssm #$i rc=$rc $(bl $o/bench_cdssm_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 bash tools/gpu_runs/dist_rehearsal.sh > $o/rehearsal.log 2>&1
rc=$?; cat $o/rehearsal.log; [ $rc -eq 0 ] || exit $rc
exit 0
fi
for M in mlp chunked chunked_cdssm bert cdssm_char; do
timeout -k 10 400 python -u bench.py --model $M > $o/bench_$M.log 2>&1
rc=$?; echo "bench $M rc=$rc $(bl $o/bench_$M.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --model cdssm_char --dtype fp32 --batch 128 > $o/bench_cdssm_char_fp32.log 2>&1
rc=$?; echo "bench cdssm_char fp32 rc=$rc $(bl $o/bench_cdssm_char_fp32.log)"; [ $rc -eq 0 ] || exit $rc
