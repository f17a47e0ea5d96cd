#!/bin/bash
# cross-stream fix of the row-sparse exchange: the graph-vs-eager RCCL test three times, then validation (a)
set -o pipefail
D=gpurun_out/r5_sparse_fix; mkdir -p $D
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -k graph_captured -x -q -s \
    --timeout 250 --timeout-method thread -p no:cacheprovider > $D/rccl_$i.log 2>&1
  rc=$?; echo "run $i rc=$rc $(grep -E '^cdssm_sparse' $D/rccl_$i.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
bash tools/gpu_runs/r5_final.sh a
