# graph steps of the launch-bound configs with / without the side streams in the capture
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_capstreams; mkdir -p $O
for m in mlp chunked chunked_cdssm; do
  for i in 1 2; do
    for v in 0 1; do
      PAGEVEC_CAPTURE_STREAMS=$v timeout -k 10 300 python bench.py --model $m --recall 0 --quality-steps 0 > $O/${m}_cs${v}_$i.log 2>&1 || exit $?
      echo "$m cs=$v run $i $(tail -1 $O/${m}_cs${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['hip_graph'])")"
    done
  done
done
