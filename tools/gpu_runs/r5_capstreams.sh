#!/bin/bash
# hipGraph capture WITH the side streams (PAGEVEC_CAPTURE_STREAMS=1) for the CDSSM step: tests, then eager vs graph
set -o pipefail
D=gpurun_out/r5_capstreams; mkdir -p $D
PAGEVEC_CAPTURE_STREAMS=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "hipgraph" -x -q \
  --timeout 250 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $D/tests.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model cdssm --graph 0 --recall 0 --quality-steps 0 --eager-compare 0 > $D/eager_$r.log 2>&1
  rc=$?; echo "eager r$r rc=$rc $(grep '^{' $D/eager_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["hip_graph"])')"; [ $rc -eq 0 ] || exit $rc
  PAGEVEC_CAPTURE_STREAMS=1 timeout -k 10 300 python -u bench.py --model cdssm --graph 1 --recall 0 --quality-steps 0 --eager-compare 0 > $D/graphms_$r.log 2>&1
  rc=$?; echo "graph+streams r$r rc=$rc $(grep '^{' $D/graphms_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["hip_graph"])')"; [ $rc -eq 0 ] || exit $rc
done
