#!/bin/bash
# ib7 (software-pipelined loss kernel) + BERT embedding / qkv bias-grad A/Bs
set -o pipefail
mkdir -p gpurun_out/r5_ib7
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "bert or attention or new_config or inbatch" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_ib7/tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r5_ib7/tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ib_micro.py --M 16384,131072 --ib 5,7,3 > gpurun_out/r5_ib7/ib_micro.log 2>&1
rc=$?; echo "ib micro rc=$rc"; grep "M=131072" gpurun_out/r5_ib7/ib_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.transformer --flag BERT_EMBED \
  --preset bert_dp8 --rounds 4 --steps 8 > gpurun_out/r5_ib7/bert_embed_ab.txt 2>&1
rc=$?; echo "embed ab rc=$rc $(tail -1 gpurun_out/r5_ib7/bert_embed_ab.txt)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.transformer --flag ATTN_BGRAD \
  --preset bert_dp8 --rounds 4 --steps 8 > gpurun_out/r5_ib7/bert_bgrad_ab.txt 2>&1
rc=$?; echo "bgrad ab rc=$rc $(tail -1 gpurun_out/r5_ib7/bert_bgrad_ab.txt)"; exit $rc
