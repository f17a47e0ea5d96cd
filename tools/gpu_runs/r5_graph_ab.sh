#!/bin/bash
# eager vs hipGraph step for the conv-tower models (bench.py --graph 0 / 1), interleaved
set -o pipefail
D=gpurun_out/r5_graph_ab; mkdir -p $D
for r in 1 2; do
  for M in chunked_cdssm cdssm; do
    for G in 0 1; do
      timeout -k 10 300 python -u bench.py --model $M --graph $G --recall 0 --quality-steps 0 --eager-compare 0 > $D/${M}_g${G}_r$r.log 2>&1
      rc=$?; echo "$M graph=$G r$r rc=$rc $(grep '^{' $D/${M}_g${G}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["hip_graph"])')"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
