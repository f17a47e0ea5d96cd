cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do for g in 0 1; do
  timeout -k 10 300 python bench.py --graph $g --steps 30 --quality-steps 0 --recall 0 --eager-compare 0 > gpurun_out/graph_ab_$g.log 2>&1
  rc=$?; echo "graph=$g rc=$rc $(tail -1 gpurun_out/graph_ab_$g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["hip_graph"])')"
  [ $rc -eq 0 ] || exit $rc
done; done
