#!/bin/bash
# ib7 with 2-step prefetch + scalar scale multiply: loss tests, micro (gens 5 / 7 / 3), PMC pass 1
set -o pipefail
D=gpurun_out/${OUTD:-r5_ib7c}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "inbatch" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $D/tests.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ib_micro.py --M 16384,131072 --ib 5,7,3 > $D/ib_micro.log 2>&1
rc=$?; echo "ib micro rc=$rc"; grep "M=" $D/ib_micro.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CMD="python3 tools/ib_micro.py --M 131072 --iters 3 --ib 5,7"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $D/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > $D/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; exit $rc
