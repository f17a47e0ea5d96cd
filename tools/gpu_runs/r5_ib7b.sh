#!/bin/bash
# coalesced embed wgrad + DPP bias-grad partials: tests + step A/Bs; ib5 / ib7 PMC
set -o pipefail
D=gpurun_out/r5_ib7b; mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "bert or attention or new_config" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $D/tests.log)"; [ $rc -eq 0 ] || exit $rc
for F in BERT_EMBED ATTN_BGRAD; do
  timeout -k 10 300 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.transformer --flag $F \
    --preset bert_dp8 --rounds 4 --steps 8 > $D/ab_$F.txt 2>&1
  rc=$?; echo "$F ab rc=$rc $(tail -1 $D/ab_$F.txt)"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 tools/ib_micro.py --M 131072 --iters 3 --ib 5,7"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $D/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > $D/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $D/p2 -o p2 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_IDX_ACTIVE GRBM_COUNT -- $CMD > $D/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; exit $rc
