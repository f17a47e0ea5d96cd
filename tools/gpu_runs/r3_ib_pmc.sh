# Round 3: in-batch / cross-GPU loss kernels at the W = 8 shape (B 4096 x M 131072):
# timing (kernel trace) + PMC counters, one pass per counter group
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ibpmc
export TMPDIR=/tmp
CMD="python3 tools/ib_micro.py --M 131072 --iters 3 ${IB_ARGS}"
timeout -k 10 300 python3 tools/ib_micro.py --M 16384,131072 --iters 10 ${IB_ARGS} > gpurun_out/ibpmc/time.log 2>&1
rc=$?; cat gpurun_out/ibpmc/time.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ibpmc/kt -o kt -- $CMD > gpurun_out/ibpmc/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ibpmc/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > gpurun_out/ibpmc/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ibpmc/p2 -o p2 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_IDX_ACTIVE GRBM_COUNT -- $CMD > gpurun_out/ibpmc/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; exit $rc
