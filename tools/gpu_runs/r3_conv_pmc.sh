# Round 3: PMC of the production conv forward (v4) + sparse backward kernels at the bench shape
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cpmc
export TMPDIR=/tmp
CMD="python3 tools/conv_micro.py --variants 0 --rounds 1 --iters 3 --bwd"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cpmc/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > gpurun_out/cpmc/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cpmc/p2 -o p2 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_IDX_ACTIVE GRBM_COUNT -- $CMD > gpurun_out/cpmc/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cpmc/p3 -o p3 --pmc TCC_HIT_sum TCC_MISS_sum -- $CMD > gpurun_out/cpmc/p3.log 2>&1
rc=$?; echo "p3 rc=$rc"; exit $rc
