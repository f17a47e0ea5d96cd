# query tower before the page tower (PAGEVEC_QUERY_FIRST) A/B, alternated in separate processes on one box
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_qfirst
for r in 1 2 3; do for Q in 0 1; do
PAGEVEC_QUERY_FIRST=$Q timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --quality-steps 0 --recall 0 --eager-compare 0 > gpurun_out/r4_qfirst/q${Q}_$r.log 2>&1
rc=$?; echo "Q=$Q run $r rc=$rc $(grep '^{' gpurun_out/r4_qfirst/q${Q}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; [ $rc -eq 0 ] || exit $rc
done; done
