# capture with side streams (query stream + page early sort, no nested fork): the hipgraph test,
# then bench eager vs graph alternated
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_capstreams; mkdir -p $O
PAGEVEC_CAPTURE_STREAMS=1 timeout -k 10 240 python -X faulthandler -u -m pytest tests/test_kernels_gpu.py -k "hipgraph" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/nonested.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/nonested.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --graph 0 --recall 0 --quality-steps 0 --eager-compare 0 > $O/eager_$i.log 2>&1 || exit $?
  PAGEVEC_CAPTURE_STREAMS=1 timeout -k 10 300 python bench.py --graph 1 --recall 0 --quality-steps 0 --eager-compare 0 > $O/graph_$i.log 2>&1 || exit $?
  echo "eager $(tail -1 $O/eager_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['hip_graph'])")  graph+streams $(tail -1 $O/graph_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['hip_graph'], d['graph_status'])")"
done
