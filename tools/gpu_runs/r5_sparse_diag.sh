#!/bin/bash
set -o pipefail
D=gpurun_out/r5_sparse_diag; mkdir -p $D
timeout -k 10 240 python -u tools/sparse_graph_diag.py --runs e,e,e,g,g > $D/diag_qs1.log 2>&1
rc=$?; cat $D/diag_qs1.log | grep "^run"; [ $rc -eq 0 ] || exit $rc
PAGEVEC_QUERY_STREAM=0 timeout -k 10 240 python -u tools/sparse_graph_diag.py --runs e,e,e,g > $D/diag_qs0.log 2>&1
rc=$?; cat $D/diag_qs0.log | grep "^run"; exit $rc
