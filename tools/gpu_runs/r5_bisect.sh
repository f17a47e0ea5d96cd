#!/bin/bash
# graph-vs-eager RCCL test under loss generations 5 and 7, then the ib8 loss run
set -o pipefail
D=gpurun_out/r5_bisect; mkdir -p $D
for G in 5 7; do
  PAGEVEC_IB=$G timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -k graph_captured -x -q -s \
    --timeout 250 --timeout-method thread -p no:cacheprovider > $D/rccl_ib$G.log 2>&1
  echo "IB=$G rc=$? $(grep -E '^(mlp|cdssm)' $D/rccl_ib$G.log | tr '\n' ' ')"
done
OUTD=r5_ib8 bash tools/gpu_runs/r5_ib7c.sh
